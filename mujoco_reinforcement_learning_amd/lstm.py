"""Windowed BiLSTM actor-critic on the MI355X engine.

The reference's ``PPOAgent`` binds ``models.lstm.lstm_actor.LSTMActor`` and
``models.lstm.lstm_critic.LSTMCritic`` (entities/agents/ppo_agent.py:2-3); this module is that
agent on the gfx950 kernels of ``csrc/bilstm.hip`` (C-ABI ``ppo_lstm_*``):

  * ``LSTMEngine``      the ``ppo_lstm_ctx`` front end, with the ``Engine`` methods the PPO loop
                        calls (``policy_step``, ``observe_act``, ``minibatch_grad``), so
                        ``PPOEngine`` trains it unchanged;
  * ``EngineLSTMActor`` / ``EngineLSTMCritic``  parameter skeletons with the reference's module
                        structure and state_dict keys (``feature_extractor.weight_ih_l0``,
                        ``actor.first_layers.0.weight``, ``actor_logstd.last_layer.bias``,
                        ``feature_extractor.0.weight_hh_l0_reverse``, ``network.*``), initialised in
                        the reference's RNG order (lstm_actor.py:12-38, lstm_critic.py:19-31);
  * ``LSTMEngineAgent`` the PPOAgent surface (act / get_state_value / optimizers / save / load).

The actor's std is per row, (B, A) = 0.2 * exp(tanh(MLP_ls(features))): the reference's
``torch.repeat_interleave(std[None, :], B, dim=0)`` (lstm_actor.py:48) turns it into (B, B, A),
which ``torch.distributions.Normal`` cannot pair with the (B, A) mean -- the
engine implements the per-row std that line means.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch
from torch import nn

from . import _lib
from . import engine as E
from ._lib import check, ptr
from .agent import _ACT_NAMES, ExponentialLRFacade, FlatAdam, PPOEngineAgent
from .engine import _need, _stream
from .features import Run
from .models import _Block, move_to_flat


class LSTMEngine:
    """One ``ppo_lstm_ctx``: BiLSTM actor + critic shapes, workspace and split-K slabs."""

    fused = False  # the layered path: no bf16 weight images, no staged records

    def __init__(self, obs_dim: int, window: int, act_dim: int, latent: int, actor_layers: int,
                 hidden, activation: str = "relu", use_bias: bool = True,
                 max_rows: int = 4096, device: Optional[torch.device] = None):
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        cfg = _lib.LstmCfg()
        cfg.obs_dim, cfg.window, cfg.act_dim = obs_dim, window, act_dim
        cfg.activation = _lib.ACT_CODES[activation]
        cfg.use_bias = int(bool(use_bias))
        cfg.latent, cfg.actor_layers = int(latent), int(actor_layers)
        cfg.n_hidden = len(hidden)
        for i, h in enumerate(hidden):
            cfg.hidden[i] = int(h)
        cfg.max_rows = int(max_rows)
        self.cfg = cfg
        self.obs_dim, self.window, self.act_dim, self.latent = obs_dim, window, act_dim, latent
        self.in_dim = obs_dim * window
        self.max_rows = int(max_rows)
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self.lib.ppo_lstm_ctx_create(ctypes.byref(cfg), self.device.index or 0,
                                               ctypes.byref(handle)))
        self._ctx = handle
        total, n_actor = ctypes.c_int64(), ctypes.c_int64()
        n = self.lib.ppo_lstm_param_layout(self._ctx, None, 0, ctypes.byref(total),
                                           ctypes.byref(n_actor))
        check(min(n, 0))
        arr = (ctypes.c_int64 * n)()
        self.lib.ppo_lstm_param_layout(self._ctx, arr, n, None, None)
        self._offsets = list(arr)
        self.n_params, self.n_actor = int(total.value), int(n_actor.value)
        self.n_critic = self.n_params - self.n_actor
        self.precision = "f32"
        self._params = None

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and ctx.value:
            try:
                self.lib.ppo_lstm_ctx_destroy(ctx)
            except Exception:  # interpreter shutdown
                pass
            self._ctx = None

    def param_offsets(self) -> list:
        return list(self._offsets)

    def bind(self, flat_params: torch.Tensor) -> None:
        _need(flat_params, "flat_params", torch.float32, (self.n_params,), self.device)
        check(self.lib.ppo_lstm_bind_params(self._ctx, ptr(flat_params)))
        self._params = flat_params

    def loss_entropy_share(self, share: float) -> None:
        """Share of the entropy bonus in the LOGGED actor loss (ppo_lstm_loss_entropy_share)."""
        check(self.lib.ppo_lstm_loss_entropy_share(self._ctx, float(share)))

    def set_precision(self, precision: str) -> None:
        if precision not in _lib.PREC_CODES:
            raise ValueError(f"unknown precision {precision!r}; use one of {sorted(_lib.PREC_CODES)}")
        check(self.lib.ppo_lstm_set_precision(self._ctx, _lib.PREC_CODES[precision]))
        self.precision = precision

    def pack_weights(self) -> None:
        """No bf16 weight images on this path."""

    def _check_state(self, state: torch.Tensor) -> int:
        n = state.shape[0]
        _need(state, "state", torch.float32, device=self.device)
        if state.numel() != n * self.in_dim:
            raise RuntimeError(f"state has {state.numel() // max(n, 1)} features per row, "
                               f"expected W*O={self.in_dim}")
        return n

    def forward(self, state: torch.Tensor, mean=None, std=None, value=None, actor_lstm_out=None,
                critic_lstm_out=None) -> None:
        """LSTMActor.forward + LSTMCritic.forward (lstm_actor.py:41-48, lstm_critic.py:33-41)."""
        n = self._check_state(state)
        for name, t, k in (("mean", mean, self.act_dim), ("std", std, self.act_dim),
                           ("value", value, 1),
                           ("actor_lstm_out", actor_lstm_out, self.window * 2 * self.latent),
                           ("critic_lstm_out", critic_lstm_out, self.window * 2 * self.latent)):
            if t is not None:
                _need(t, name, torch.float32, device=self.device)
                if t.numel() != n * k:
                    raise RuntimeError(f"{name} has {t.numel()} elements, expected {n * k}")
        check(self.lib.ppo_lstm_forward(self._ctx, ptr(state), n, ptr(mean), ptr(std), ptr(value),
                                        ptr(actor_lstm_out), ptr(critic_lstm_out),
                                        _stream(self.device)))

    def policy_step(self, state: torch.Tensor, eps: Optional[torch.Tensor] = None, seed: int = 0,
                    offset: int = 0, action=None, logp=None, value=None, mean=None) -> None:
        """ppo.py:22-26 for one rollout step (the ``Engine.policy_step`` contract)."""
        n = self._check_state(state)
        if mean is not None:
            self.forward(state, mean=mean)
            if action is None and value is None:
                return
        if eps is not None:
            _need(eps, "eps", torch.float32, (n, self.act_dim), self.device)
        for name, t, k in (("action", action, self.act_dim), ("logp", logp, 1), ("value", value, 1)):
            if t is not None:
                _need(t, name, torch.float32, device=self.device)
                if t.numel() != n * k:
                    raise RuntimeError(f"{name} has {t.numel()} elements, expected {n * k}")
        check(self.lib.ppo_lstm_policy_step(self._ctx, ptr(state), n, ptr(eps), seed, offset,
                                            ptr(action), ptr(logp), ptr(value),
                                            _stream(self.device)))

    def observe_act(self, window: torch.Tensor, state: torch.Tensor, obs=None, reset=None,
                    all_reset: bool = False, normalize: bool = True, eps=None, seed: int = 0,
                    offset: int = 0, action=None, logp=None, value=None, mean=None) -> None:
        """Window push + standardisation (ppo_obs_window_push / ppo_obs_normalize), then the
        LSTM policy step: the ``Engine.observe_act`` contract."""
        if obs is not None:
            E.obs_window_push(window, obs, reset, all_reset)
        E.obs_normalize(window, state, normalize)
        self.policy_step(state.reshape(state.shape[0], -1), eps=eps, seed=seed, offset=offset,
                         action=action, logp=logp, value=value, mean=mean)

    def minibatch_grad(self, states, actions, old_logp, adv, vtarget, rows, b: int, grad, loss,
                       clip_lo: float, clip_hi: float, entropy_coef: float, inv_b: float,
                       inv_ba: float, count: Optional[torch.Tensor] = None) -> None:
        """ppo.py:108-135 for one minibatch (the ``Engine.minibatch_grad`` contract)."""
        if count is not None:
            raise NotImplementedError("the LSTM agent runs the single-process / local-DP paths")
        _need(rows, "rows", torch.int32, device=self.device)
        _need(grad, "grad", torch.float32, (self.n_params,), self.device)
        if loss is not None:
            _need(loss, "loss", torch.float32, device=self.device)
        check(self.lib.ppo_lstm_minibatch_grad(
            self._ctx, ptr(states), ptr(actions), ptr(old_logp), ptr(adv), ptr(vtarget),
            ptr(rows), int(b), ptr(grad), ptr(loss), clip_lo, clip_hi, entropy_coef, inv_b,
            inv_ba, _stream(self.device)))

    def fused_step(self, enable: Optional[bool] = None) -> bool:
        """bf16 forward steps as one recurrent-GEMM + cell launch (ppo_lstm_fused_step); set it
        with enable, return the current setting."""
        if enable is not None:
            check(self.lib.ppo_lstm_fused_step(self._ctx, int(bool(enable))))
        return bool(self.lib.ppo_lstm_fused_step(self._ctx, -1))

    # ---- measurement (the Engine.timing* contract of bench.py) ----------------------------------
    def timing(self, enable: bool, capacity: int = 65536) -> None:
        check(self.lib.ppo_lstm_timing(self._ctx, int(enable), int(capacity)))

    def timing_kernels(self) -> dict:
        out = {}
        n_k = self.lib.ppo_lstm_timing_kernel(self._ctx, -1, None, None, None, None, None, None)
        check(min(n_k, 0))
        for i in range(n_k):
            name, cls = ctypes.c_char_p(), ctypes.c_int()
            ms, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
            cnt = ctypes.c_int64()
            check(self.lib.ppo_lstm_timing_kernel(self._ctx, i, ctypes.byref(name),
                                                  ctypes.byref(cls), ctypes.byref(ms),
                                                  ctypes.byref(cnt), ctypes.byref(fl),
                                                  ctypes.byref(by)))
            out[name.value.decode()] = {
                "class": self.lib.ppo_kernel_class_name(cls.value).decode(), "ms": ms.value,
                "launches": cnt.value, "flops": fl.value, "bytes": by.value}
        return out

    def timing_read(self) -> dict:
        out = {}
        for name, k in self.timing_kernels().items():
            c = out.setdefault(k["class"], {"ms": 0.0, "launches": 0, "flops": 0.0, "bytes": 0.0})
            for key in ("ms", "launches", "flops", "bytes"):
                c[key] += k[key]
        return out


class EngineLSTMActor(nn.Module):
    """models/lstm/lstm_actor.py:9-38 (parameters only; forward through the engine)."""

    def __init__(self, obs_dim: int, latent: int, layers: int, window: int, hidden, act_dim: int,
                 act_cls, use_bias: bool, last_layer_std: float):
        super().__init__()
        # nn.LSTM is the parameter container (its reset_parameters draws the reference's RNG)
        self.feature_extractor = nn.LSTM(obs_dim, latent, num_layers=layers, bidirectional=True,
                                         batch_first=True)
        in_dim = latent * 2 * window
        self.actor = _Block(in_dim, hidden, act_dim, act_cls, use_bias, last_layer_std)
        self.actor_logstd = _Block(in_dim, hidden, act_dim, act_cls, use_bias, last_layer_std)
        self._agent = None

    def forward(self, x):
        return self._agent._actor_mean_std(x)


class EngineLSTMCritic(nn.Module):
    """models/lstm/lstm_critic.py:9-31 (parameters only; forward through the engine)."""

    def __init__(self, obs_dim: int, latent: int, hidden, act_cls, use_bias: bool,
                 last_layer_std: float):
        super().__init__()
        self.feature_extractor = nn.Sequential(
            nn.LSTM(obs_dim, latent, bidirectional=True, batch_first=True))
        self.network = _Block(latent * 2, hidden, 1, act_cls, use_bias, last_layer_std)
        self._agent = None

    def forward(self, x):
        return self._agent.get_state_value(x)


class LSTMEngineAgent(PPOEngineAgent):
    """PPOAgent with the reference's LSTM actor / critic (ppo_agent.py:10-43) on the engine."""

    def __init__(self, run: Optional[Run] = None, device: Optional[torch.device] = None,
                 max_rows: Optional[int] = None):
        run = run or Run.instance()
        if run is None:
            raise ValueError("LSTMEngineAgent needs a Run (construct entities Run first)")
        self.run = run
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        nc, ec = run.network_config, run.environment_config
        act_cls = nc.activation_class
        if act_cls not in _ACT_NAMES:
            raise ValueError(f"activation {act_cls} not supported by the engine (ReLU/Tanh/ELU)")
        hidden = list(nc.linear_hidden_shapes)[:nc.num_linear_layers]
        latent, layers = int(nc.feature_extractor_latent_size), int(nc.num_feature_extractor_layers)
        self.networks = nn.ModuleDict()
        # PPOAgent.initialize_networks: Actor() then Critic() (RNG order)
        self.networks["actor"] = EngineLSTMActor(nc.input_shape, latent, layers,
                                                 ec.window_length, hidden, nc.output_shape,
                                                 act_cls, nc.use_bias, nc.last_layer_std)
        self.networks["critic"] = EngineLSTMCritic(nc.input_shape, latent, hidden, act_cls,
                                                   nc.use_bias, nc.last_layer_std)
        for m in (self.networks["actor"], self.networks["critic"]):
            m._agent = self
        rows = max_rows or max(ec.num_envs, int(run.training_config.batch_size))
        self.engine = LSTMEngine(nc.input_shape, ec.window_length, nc.output_shape, latent, layers,
                                 hidden, _ACT_NAMES[act_cls], nc.use_bias, rows, self.device)
        self.flat_params = move_to_flat(self.networks, self.device, self.engine.param_offsets(),
                                        self.engine.n_params)
        for mod in self.networks.modules():  # keep nn.LSTM's flat-weight list on the views
            if isinstance(mod, nn.LSTM):
                mod._init_flat_weights()
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

    def _actor_mean_std(self, state: torch.Tensor):
        s = self._as_state(state)
        n, a = len(s), self.engine.act_dim
        mean = torch.empty(n, a, device=self.device)
        std = torch.empty(n, a, device=self.device)
        self.engine.forward(s, mean=mean, std=std)
        return mean, std

    def _actor_mean(self, state: torch.Tensor) -> torch.Tensor:
        return self._actor_mean_std(state)[0]

    def get_state_value(self, state: torch.Tensor) -> torch.Tensor:
        """ppo_agent.py:24-25 -> (n, 1)."""
        s = self._as_state(state)
        value = torch.empty(len(s), 1, device=self.device)
        self.engine.forward(s, value=value)
        return value

    def act(self, state: torch.Tensor, return_dist: bool = False, test_phase: bool = False):
        """ppo_agent.py:27-43 with the per-row std of the LSTM actor."""
        s = self._as_state(state)
        n, a = len(s), self.engine.act_dim
        mean, std = self._actor_mean_std(s)
        if test_phase:
            action = mean.reshape(-1)  # torch.cat([means[i] for i in range(n)])
        else:
            action = torch.empty(n, a, device=self.device)
            if self.run.engine_config.rng == "torch":
                eps = torch.randn(n, a).to(self.device)
                self.engine.policy_step(s, eps=eps, action=action)
            else:
                self._act_offset = getattr(self, "_act_offset", 0)
                self.engine.policy_step(s, seed=self.run.engine_config.seed ^ 0x5EED,
                                        offset=self._act_offset, action=action)
                self._act_offset += n * a
        if return_dist:
            return action, torch.distributions.Normal(mean, std, validate_args=False)
        return action
