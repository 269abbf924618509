"""``PPOEngineAgent`` -- drop-in for the reference ``PPOAgent`` (ppo_agent.py:10-43, agent.py:14-72).

Same surface: ``networks`` (ModuleDict 'actor'/'critic' with the reference state_dict keys),
``optimizers`` / ``schedulers`` dicts with the same keys, ``act(state, return_dist, test_phase)``,
``get_state_value(state)``, ``save()``, ``load()``.  Parameters, gradients and Adam moments are
flat fp32 device buffers; the fused Adam kernel (ppo_adam) updates both networks in one launch.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch
from torch import nn

from . import engine as E
from .features import REFERENCE_CRITIC_HIDDEN, Run
from .models import EngineActor, EngineCritic, move_to_flat

ENGINE_RNG_FILE = "engine_rng_rank{rank}.pth"  # the per-rank torch generator of local data parallelism
LEGACY_ENGINE_RNG_FILE = "engine_rng.pth"      # round-3 name (one file, holding its rank)


def _dist_rank() -> int:
    """This process's torch.distributed rank (0 when not initialised)."""
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_rank()
    return 0

_ACT_NAMES = {nn.ReLU: "relu", nn.Tanh: "tanh", nn.ELU: "elu"}


class FlatAdam:
    """``torch.optim.Adam`` facade over one segment of the engine's flat buffers.

    ``step()`` runs the HIP Adam kernel on this segment with the scalars computed in double
    exactly as adam.py ``_single_tensor_adam`` does; ``state_dict()`` / ``load_state_dict()`` use
    torch's Adam format so optimizer_<name>.pth files interoperate with the reference.
    """

    def __init__(self, params, flat_p, flat_g, flat_m, flat_v, lo: int, hi: int, lr: float,
                 betas=(0.9, 0.999), eps: float = 1e-8):
        self.params = list(params)
        self.lo, self.hi = lo, hi
        self._p, self._g, self._m, self._v = (flat_p[lo:hi], flat_g[lo:hi], flat_m[lo:hi],
                                              flat_v[lo:hi])
        self.param_groups = [{"lr": lr, "betas": betas, "eps": eps, "weight_decay": 0,
                              "amsgrad": False, "maximize": False, "foreach": None,
                              "capturable": False, "differentiable": False, "fused": None,
                              "initial_lr": lr}]
        self.step_count = 0

    @property
    def lr(self) -> float:
        return self.param_groups[0]["lr"]

    def scalars(self, step: int):
        """(neg_step_size, bc2_sqrt) for Adam step ``step`` (adam.py, python double math)."""
        beta1, beta2 = self.param_groups[0]["betas"]
        bias_correction1 = 1 - beta1 ** step
        bias_correction2 = 1 - beta2 ** step
        step_size = self.lr / bias_correction1
        return -step_size, bias_correction2 ** 0.5

    def zero_grad(self, set_to_none: bool = True):
        self._g.zero_()

    def step(self):
        self.step_count += 1
        beta1, beta2 = self.param_groups[0]["betas"]
        neg, bc2 = self.scalars(self.step_count)
        n = self.hi - self.lo
        E.adam(self._p, self._g, self._m, self._v, n, neg, neg, 1 - beta1, beta2, 1 - beta2, bc2,
               self.param_groups[0]["eps"])

    def _views(self):
        base = self._p.data_ptr()
        for p in self.params:  # each parameter is a view of the flat buffer (padded layout)
            off = (p.data_ptr() - base) // p.element_size()
            n = p.numel()
            yield p, self._m[off:off + n].view(p.shape), self._v[off:off + n].view(p.shape)

    def state_dict(self):
        state = {}
        if self.step_count > 0:
            for i, (_, m, v) in enumerate(self._views()):
                state[i] = {"step": torch.tensor(float(self.step_count)), "exp_avg": m.clone(),
                            "exp_avg_sq": v.clone()}
        group = dict(self.param_groups[0])
        group["params"] = list(range(len(self.params)))
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        group = sd["param_groups"][0]
        for k in ("lr", "betas", "eps", "initial_lr"):
            if k in group:
                self.param_groups[0][k] = group[k]
        st = sd.get("state", {})
        if not st:
            self.step_count = 0
            self._m.zero_()
            self._v.zero_()
            return
        for i, (_, m, v) in enumerate(self._views()):
            s = st[i] if i in st else st[str(i)]
            m.copy_(s["exp_avg"].to(m.device))
            v.copy_(s["exp_avg_sq"].to(v.device))
            self.step_count = int(float(s["step"]))


class ExponentialLRFacade:
    """``torch.optim.lr_scheduler.ExponentialLR`` (gamma per ``step()``, chainable form)."""

    def __init__(self, optimizer: FlatAdam, gamma: float):
        self.optimizer = optimizer
        self.gamma = gamma
        self.last_epoch = 0

    def step(self):
        self.last_epoch += 1
        for g in self.optimizer.param_groups:
            g["lr"] = g["lr"] * self.gamma

    def get_last_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self):
        return {"gamma": self.gamma, "last_epoch": self.last_epoch}

    def load_state_dict(self, sd):
        self.gamma = sd["gamma"]
        self.last_epoch = sd["last_epoch"]


def make_agent(run: Optional[Run] = None, device: Optional[torch.device] = None,
               max_rows: Optional[int] = None):
    """The agent NetworkConfig.feature_extractor selects: "LSTM" -> the reference PPOAgent's
    LSTM actor / critic (ppo_agent.py:2-3; lstm.LSTMEngineAgent), "CNN" -> the pixel actor /
    critic of BASELINE configs[4] (cnn.CNNEngineAgent), anything else -> the MLP actor-critic of
    north_star (PPOEngineAgent)."""
    run = run or Run.instance()
    kind = str(getattr(run.network_config, "feature_extractor", "MLP")).upper()
    if kind == "LSTM":
        from .lstm import LSTMEngineAgent
        return LSTMEngineAgent(run, device, max_rows)
    if kind == "CNN":  # pixel observations (BASELINE configs[4]; cnn.py)
        from .cnn import CNNEngineAgent
        return CNNEngineAgent(run, device, max_rows)
    return PPOEngineAgent(run, device, max_rows)


class PPOEngineAgent:
    """PPOAgent on the MI355X engine."""

    def __init__(self, run: Optional[Run] = None, device: Optional[torch.device] = None,
                 max_rows: Optional[int] = None):
        run = run or Run.instance()
        if run is None:
            raise ValueError("PPOEngineAgent needs a Run (construct entities Run first)")
        self.run = run
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        nc, ec = run.network_config, run.environment_config
        act_cls = nc.activation_class
        if act_cls not in _ACT_NAMES:
            raise ValueError(f"activation {act_cls} not supported by the engine (ReLU/Tanh/ELU)")
        hidden = list(nc.linear_hidden_shapes)[:nc.num_linear_layers]
        # models/critic.py:10-15 hard-codes [128, 128]; engine_config may widen it
        critic_hidden = list(run.engine_config.critic_hidden_shapes or REFERENCE_CRITIC_HIDDEN)
        in_dim = nc.input_shape * ec.window_length
        self.networks = nn.ModuleDict()
        # PPOAgent.initialize_networks builds the actor first, then the critic (RNG order)
        self.networks["actor"] = EngineActor(in_dim, hidden, nc.output_shape, act_cls,
                                             nc.use_bias, nc.output_max_value)
        self.networks["critic"] = EngineCritic(in_dim, critic_hidden, act_cls)
        for m in (self.networks["actor"], self.networks["critic"]):
            m._agent = self
        rows = max_rows or max(ec.num_envs, int(run.training_config.batch_size))
        self.engine = E.Engine(nc.input_shape, ec.window_length, nc.output_shape, hidden,
                               critic_hidden, _ACT_NAMES[act_cls], nc.use_bias,
                               nc.output_max_value, rows, self.device)
        self.flat_params = move_to_flat(self.networks, self.device, self.engine.param_offsets(),
                                        self.engine.n_params)
        self.engine.bind(self.flat_params)
        self.engine.set_precision(getattr(run.engine_config, "precision", "f32"))
        self.flat_grad = torch.zeros_like(self.flat_params)
        self.flat_m = torch.zeros_like(self.flat_params)
        self.flat_v = torch.zeros_like(self.flat_params)
        na = self.engine.n_actor
        lr = run.training_config.learning_rate
        self.optimizers: Dict[str, FlatAdam] = {
            "actor": FlatAdam(self.networks["actor"].parameters(), self.flat_params,
                              self.flat_grad, self.flat_m, self.flat_v, 0, na, lr),
            "critic": FlatAdam(self.networks["critic"].parameters(), self.flat_params,
                               self.flat_grad, self.flat_m, self.flat_v, na,
                               self.engine.n_params, lr),
        }
        self.schedulers = {k: ExponentialLRFacade(o, 0.999) for k, o in self.optimizers.items()}

    def packed_params(self) -> torch.Tensor:
        """All parameters concatenated in parameters() order (no alignment padding)."""
        return torch.cat([p.detach().reshape(-1) for p in self.networks.parameters()])

    def packed(self, flat: torch.Tensor) -> torch.Tensor:
        """Any flat-layout buffer (grad, m, v) gathered into parameters() order."""
        base = self.flat_params.data_ptr()
        out = []
        for p in self.networks.parameters():
            off = (p.data_ptr() - base) // 4
            out.append(flat[off:off + p.numel()])
        return torch.cat(out)

    # ---- fused optimizer step for both networks (ppo.py:122 + :135 in one launch) -------------
    def step_both(self, pack: bool = False) -> bool:
        """One Adam step of both optimizers in one launch.  pack=True (fused bf16 engine) also
        refreshes the fused kernels' bf16 weight images (ppo_adam_pack); returns whether the
        images are current afterwards."""
        oa, oc = self.optimizers["actor"], self.optimizers["critic"]
        oa.step_count += 1
        oc.step_count += 1
        beta1, beta2 = oa.param_groups[0]["betas"]
        neg_a, bc2 = oa.scalars(oa.step_count)
        neg_c, bc2c = oc.scalars(oc.step_count)
        if (bc2 != bc2c or oc.param_groups[0]["betas"] != (beta1, beta2) or
                oc.param_groups[0]["eps"] != oa.param_groups[0]["eps"]):
            oa.step_count -= 1
            oc.step_count -= 1
            oa.step()
            oc.step()
            return False
        eps = oa.param_groups[0]["eps"]
        if pack:
            self.engine.adam_pack(self.flat_grad, self.flat_m, self.flat_v, None, neg_a, neg_c, bc2,
                                  1 - beta1, beta2, 1 - beta2, eps)
            return True
        E.adam(self.flat_params, self.flat_grad, self.flat_m, self.flat_v, self.engine.n_actor,
               neg_a, neg_c, 1 - beta1, beta2, 1 - beta2, bc2, eps)
        return False

    def adam_schedule(self, steps: int):
        """Host-computed Adam scalars for the next ``steps`` joint steps of both optimizers, as an
        (steps, 4) f32 tensor of (neg_step_actor, neg_step_critic, bc2_sqrt, 0) rows (the values
        step_both would pass to ppo_adam), advancing both step counters; None when the two
        optimizers' hyper-parameters differ (then step_both's per-net path is required)."""
        oa, oc = self.optimizers["actor"], self.optimizers["critic"]
        ga, gc = oa.param_groups[0], oc.param_groups[0]
        if ga["betas"] != gc["betas"] or ga["eps"] != gc["eps"] or oa.step_count != oc.step_count:
            return None
        rows = []
        for k in range(oa.step_count + 1, oa.step_count + steps + 1):
            neg_a, bc2 = oa.scalars(k)
            neg_c, bc2c = oc.scalars(k)
            if bc2 != bc2c:
                return None
            rows.append((neg_a, neg_c, bc2, 0.0))
        oa.step_count += steps
        oc.step_count += steps
        return torch.tensor(rows, dtype=torch.float32)

    # ---- Agent API ---------------------------------------------------------------------------
    def _as_state(self, state: torch.Tensor) -> torch.Tensor:
        s = state.to(device=self.device, dtype=torch.float32)
        return s.reshape(len(s), -1).contiguous()

    def _actor_mean(self, state: torch.Tensor) -> torch.Tensor:
        s = self._as_state(state)
        mean = torch.empty(len(s), self.engine.act_dim, device=self.device)
        self.engine.policy_step(s, mean=mean)
        return mean

    def get_state_value(self, state: torch.Tensor) -> torch.Tensor:
        """ppo_agent.py:24-25 -> (n, 1)."""
        s = self._as_state(state)
        value = torch.empty(len(s), 1, device=self.device)
        self.engine.policy_step(s, value=value)
        return value

    def act(self, state: torch.Tensor, return_dist: bool = False, test_phase: bool = False):
        """ppo_agent.py:27-43.  Sampling noise: torch global CPU generator (rng="torch", the
        reference's ``Normal.sample`` draws) or on-device Philox (rng="philox")."""
        s = self._as_state(state)
        n, a = len(s), self.engine.act_dim
        mean = torch.empty(n, a, device=self.device)
        std = self.networks["actor"].actor_logstd.detach().exp()
        if test_phase:
            self.engine.policy_step(s, mean=mean)
            action = mean.reshape(-1)  # torch.cat([means[i] for i in range(n)])
        else:
            action = torch.empty(n, a, device=self.device)
            if self.run.engine_config.rng == "torch":
                eps = torch.randn(n, a).to(self.device)
                self.engine.policy_step(s, eps=eps, action=action, mean=mean)
            else:
                self._act_offset = getattr(self, "_act_offset", 0)
                self.engine.policy_step(s, seed=self.run.engine_config.seed ^ 0x5EED,
                                        offset=self._act_offset, action=action, mean=mean)
                self._act_offset += n * a
        if return_dist:
            dist = torch.distributions.Normal(mean, std[None, :].expand(n, a), validate_args=False)
            return action, dist
        return action

    # ---- checkpoint (agent.py:47-72; same files and keys) ------------------------------------
    def save(self):
        run = Run.instance()
        path = f"{run.experiment_path}/networks/{run.dynamic_config.current_episode}"
        os.makedirs(path, exist_ok=True)
        torch.save({k: v.detach().cpu() for k, v in self.networks.state_dict().items()},
                   f"{path}/networks.pth")
        for name, opt in self.optimizers.items():
            sd = opt.state_dict()
            sd["state"] = {i: {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in s.items()}
                           for i, s in sd["state"].items()}
            torch.save(sd, f"{path}/optimizer_{name}.pth")
        algo = getattr(self, "_algorithm", None)
        state = algo.rng_state() if algo is not None else None
        if state is not None:  # engine-only file (one per rank): the reference never reads it
            torch.save(state, f"{path}/{ENGINE_RNG_FILE.format(rank=state['rank'])}")
        run.save()

    def load(self):
        run = Run.instance()
        base = run.experiment_path
        ep = run.dynamic_config.current_episode
        path = f"{base}/networks/{ep}"
        if not os.path.exists(path):
            path = f"{base}/networks/best_results/{ep}"
        if not os.path.exists(path):
            raise ValueError("the current iteration does not exist")
        sd = torch.load(f"{path}/networks.pth", map_location="cpu", weights_only=True)
        self.networks.load_state_dict(sd)
        for name, opt in self.optimizers.items():
            opt.load_state_dict(torch.load(f"{path}/optimizer_{name}.pth", map_location="cpu",
                                           weights_only=True))
        algo = getattr(self, "_algorithm", None)
        rank = algo.dp.rank if algo is not None else _dist_rank()
        rng_file = f"{path}/{ENGINE_RNG_FILE.format(rank=rank)}"
        state = torch.load(rng_file, weights_only=True) if os.path.exists(rng_file) else None
        legacy = f"{path}/{LEGACY_ENGINE_RNG_FILE}"
        if state is None and os.path.exists(legacy):
            # a checkpoint written before the per-rank files: use it when it holds this rank's
            # generator, otherwise say that this rank continues from a fresh seed
            old = torch.load(legacy, weights_only=True)
            if isinstance(old, dict) and old.get("rank") == rank:
                state = old
            else:
                import warnings
                warnings.warn(f"{legacy} holds rank {old.get('rank') if isinstance(old, dict) else '?'}'s "
                              f"generator; rank {rank} continues from a freshly seeded one",
                              stacklevel=2)
        if algo is not None:
            algo.set_rng_state(state)
        else:
            # the reference's order builds the agent, loads, then builds the trainer: keep the
            # state for PPOEngine.__init__ to pick up
            self._loaded_rng_state = state
