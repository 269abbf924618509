"""CPU oracle for the PPO rollout -> GAE -> update hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline``
leg of ``bench.py`` may import this module, and only as the checker / the timed CPU baseline.
The product package (``mujoco_reinforcement_learning_amd``) never imports it and never falls back
to it.

What it restates (reference = aminrezaee/mujoco_reinforcement_learning @ 2025-03-03):

* ``MLPBlock``            network_block_creator.py:18-86 (orthogonal sqrt(2) hidden init with zero
                          bias, orthogonal 0.01 last layer with the default ``Linear`` bias init)
* ``RefActor``            models/linear/actor.py:9-32 (flatten window, tanh head, x output_max_value,
                          state-independent ``actor_logstd``)
* ``RefCritic``           models/critic.py:6-25 with the window flattened exactly like the actor
                          (the reference critic has no flatten and returns (N,W,1))
* ``RefAgent``            entities/agents/ppo_agent.py:10-43 + agent.py:26-42
* ``normalize_state``     environments/humanoid/running_gym_sequential_vectorized.py:61-92
* ``generalized_advantage_estimate``
                          torchrl 0.6.0 ``torchrl/objectives/value/functional.py`` (third-party,
                          pinned in requirements.txt:7, absent from /root/reference and from this
                          image) -- restated from its published algorithm; call site ppo.py:76-80
* ``rollout`` / ``calculate_advantages`` / ``train``
                          entities/algorithms/ppo.py:13-159

Parity pinning (see DESIGN.md "Oracle"): the MLP init + forward rows are pinned against the
reference modules themselves (tests/golden/gen_golden.py imports /root/reference/src and writes
tests/golden/reference_mlp.npz).  ``entities.algorithms.ppo`` is not importable here (tensordict,
torchrl, cv2, mlflow are missing) and the reference ships no tests or golden vectors, so the GAE
and the loss/update rows are pinned only by hand-derived known answers: **parity unpinned**
against the real torchrl / tensordict.

RNG contract (what makes a fixed-seed comparison with the engine possible): everything draws from
the torch *global* CPU generator in the reference order -- per rollout step one ``Normal.sample``
of (N, A) normals (ppo.py:23-25), then per epoch ``torch.randperm(N*T)`` (ppo.py:103) followed by
one wasted (B, A) ``Normal.sample`` per minibatch (ppo.py:110 -> ppo_agent.py:40).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
from torch import nn
from torch.nn.functional import huber_loss

ACTIVATIONS = {"relu": nn.ReLU, "tanh": nn.Tanh, "elu": nn.ELU}

# torchrl/objectives/value/functional.py SHAPE_ERR (the message torchrl raises on a shape mismatch)
SHAPE_ERR = ("All input tensors (value, reward and done states) must share a unique shape.")

# running_gym_sequential_vectorized.py:70-80 -- the Humanoid feature slices, applied whatever O is
HUMANOID_SLICES: Tuple[Tuple[int, Optional[int]], ...] = (
    (0, 22), (22, 45), (45, 175), (175, 253), (253, 270), (270, None))


@dataclass
class RefConfig:
    """The hyper-parameters the hot path reads from ``Run.instance()`` (features.py:17-87)."""
    num_envs: int = 8
    horizon: int = 16                 # EnvironmentConfig.maximum_timesteps
    obs_dim: int = 17                 # NetworkConfig.input_shape
    act_dim: int = 6                  # NetworkConfig.output_shape
    window: int = 1                   # EnvironmentConfig.window_length
    actor_hidden: Tuple[int, ...] = (64, 64)
    critic_hidden: Tuple[int, ...] = (64, 64)
    activation: str = "relu"
    use_bias: bool = True
    output_max_value: float = 1.0
    gamma: float = 0.99
    lmbda: float = 0.98
    clip_epsilon: float = 0.1
    entropy_eps: float = 1e-4
    advantage_scaler: float = 1.0
    normalize_advantage: bool = False
    normalize_rewards: bool = False
    normalize_observations: bool = True
    learning_rate: float = 1e-4
    epochs: int = 10
    batch_size: int = 64
    max_grad_norm: float = 1.0


# ----------------------------------------------------------------------------------------------
# Models
# ----------------------------------------------------------------------------------------------
class MLPBlock(nn.Module):
    """``NetworkBlock`` (network_block_creator.py:24-86) without batch-norm / skip connections.

    The RNG order matters for parity with a seeded reference build: each hidden ``Linear`` draws its
    default kaiming/uniform init, then ``orthogonal_(sqrt 2)`` redraws the weight and the bias is
    zeroed (:46-53); the last ``Linear`` draws its default init and ``orthogonal_(0.01)`` redraws the
    weight only (:63-65), so its bias keeps the default U(+-1/sqrt(fan_in)) draw.
    """

    def __init__(self, in_dim: int, hidden, out_dim: int, act_cls, final_act_cls, use_bias: bool,
                 last_layer_std: float = 0.01):
        super().__init__()
        mods: List[nn.Module] = []
        width = in_dim
        for h in hidden:
            lin = nn.Linear(width, h, bias=use_bias)
            with torch.no_grad():
                torch.nn.init.orthogonal_(lin.weight, np.sqrt(2))
                if use_bias:
                    lin.bias.fill_(0)
            mods.append(lin)
            mods.append(act_cls())
            width = h
        self.first_layers = nn.Sequential(*mods)
        self.last_layer = nn.Linear(width, out_dim, bias=use_bias)
        with torch.no_grad():
            torch.nn.init.orthogonal_(self.last_layer.weight, last_layer_std)
        self.last_layer_activation = final_act_cls() if final_act_cls is not None else None

    def forward(self, x):
        y = self.last_layer(self.first_layers(x))
        if self.last_layer_activation is not None:
            y = self.last_layer_activation(y)
        return y


class RefActor(nn.Module):
    """models/linear/actor.py:9-32."""

    def __init__(self, cfg: RefConfig):
        super().__init__()
        self.cfg = cfg
        self.actor = MLPBlock(cfg.obs_dim * cfg.window, cfg.actor_hidden, cfg.act_dim,
                              ACTIVATIONS[cfg.activation], nn.Tanh, cfg.use_bias)
        self.actor_logstd = nn.Parameter(torch.zeros(cfg.act_dim))

    def forward(self, x):
        x = x.reshape(len(x), -1)
        mean = self.cfg.output_max_value * self.actor(x)
        std = self.actor_logstd[:self.cfg.act_dim].exp()
        return mean, torch.repeat_interleave(std[None, :], x.shape[0], dim=0)


class RefCritic(nn.Module):
    """models/critic.py:6-25 with the (N, W, O) state flattened to (N, W*O) like the actor."""

    def __init__(self, cfg: RefConfig):
        super().__init__()
        self.network = MLPBlock(cfg.obs_dim * cfg.window, cfg.critic_hidden, 1,
                                ACTIVATIONS[cfg.activation], None, True)

    def forward(self, x):
        return self.network(x.reshape(len(x), -1))


class RefAgent:
    """PPOAgent (ppo_agent.py:10-43): actor built before critic, two Adams, two ExponentialLR."""

    def __init__(self, cfg: RefConfig):
        self.cfg = cfg
        self.networks = nn.ModuleDict()
        self.networks["actor"] = RefActor(cfg)
        self.networks["critic"] = RefCritic(cfg)
        self.optimizers = {
            k: torch.optim.Adam(self.networks[k].parameters(), lr=cfg.learning_rate)
            for k in ("actor", "critic")
        }
        self.schedulers = {
            k: torch.optim.lr_scheduler.ExponentialLR(self.optimizers[k], gamma=0.999)
            for k in ("actor", "critic")
        }

    def get_state_value(self, state):
        return self.networks["critic"](state)

    def act(self, state, return_dist: bool = False, test_phase: bool = False):
        means, stds = self.networks["actor"](state)
        dist = torch.distributions.Normal(means, stds)
        if test_phase:
            action = torch.cat([means[i] for i in range(len(state))], dim=0)
        else:
            action = dist.sample()
        if return_dist:
            return action, dist
        return action


# ----------------------------------------------------------------------------------------------
# Observation normalisation (A1)
# ----------------------------------------------------------------------------------------------
def _standardise(x: torch.Tensor) -> torch.Tensor:
    """running_gym_sequential_vectorized.py:61-66 (f64, unbiased std, std==0 -> 1)."""
    x = x - x.mean(dim=1).unsqueeze(1)
    std = x.std(dim=1).unsqueeze(1)
    std[std == 0] = 1
    x /= std
    return x


def normalize_state(state: torch.Tensor) -> torch.Tensor:
    """running_gym_sequential_vectorized.py:68-81 on a (N, O, W) f64 window."""
    for lo, hi in HUMANOID_SLICES:
        if state[:, lo:hi].shape[1] == 0:
            continue  # empty slice: the reference's ops on it are no-ops
        state[:, lo:hi] = _standardise(state[:, lo:hi])
    return state


def get_state(window: torch.Tensor, normalize: bool, dtype=torch.float32) -> torch.Tensor:
    """running_gym_sequential_vectorized.py:83-92: (N, O, W) f64 -> (N, W, O) ``Run.dtype``."""
    data = window.clone()
    if normalize:
        data = normalize_state(data)
    return data.to(dtype).permute(0, 2, 1)


# ----------------------------------------------------------------------------------------------
# Synthetic vectorised environment (harness input, same formulas as the engine's device kernel)
# ----------------------------------------------------------------------------------------------
class RefSyntheticEnv:
    """CPU restatement of the engine's synthetic VecEnv (mujoco_reinforcement_learning_amd.envs).

    Physics is out of scope for the hot path, so the harness drives the loop with
    synthetic dynamics whose next observation depends on the action, keeping the T rollout steps
    sequential:  obs' = base_obs[t+1] + 0.1 * a[:, o % A];  r = base_reward[t] - 0.01 * sum_a a^2
    (f64, sequential in a);  terminated = base_terminated[t].  The observation window follows
    EnvironmentHelper semantics (helper.py:51-67, running_gym_sequential_vectorized.py:40-59).
    """

    def __init__(self, base_obs: torch.Tensor, base_reward: torch.Tensor,
                 base_terminated: torch.Tensor, window: int, act_dim: int):
        self.base_obs = base_obs            # (T+1, N, O) f32
        self.base_reward = base_reward      # (T, N) f32
        self.base_terminated = base_terminated  # (T, N) bool
        self.W = window
        self.A = act_dim
        self.t = 0
        self.window = None
        self.reward = None
        self.terminated = None
        self.truncated = None

    def reset(self):
        self.t = 0
        first = self.base_obs[0].double()
        self.window = first[..., None].repeat(1, 1, self.W)   # helper.py:62-64
        n = first.shape[0]
        self.terminated = torch.zeros(n, dtype=torch.bool)
        self.truncated = torch.zeros(n, dtype=torch.bool)

    def step(self, action: torch.Tensor):
        t = self.t
        a = action.double()
        n, o = self.base_obs.shape[1], self.base_obs.shape[2]
        cols = torch.arange(o) % self.A
        nxt = self.base_obs[t + 1].double() + 0.1 * a[:, cols]
        ctrl = torch.zeros(n, dtype=torch.float64)
        for j in range(self.A):
            ctrl = ctrl + a[:, j] * a[:, j]
        self.reward = self.base_reward[t].double() - 0.01 * ctrl
        self.terminated = self.base_terminated[t].clone()
        self.truncated = torch.zeros(n, dtype=torch.bool)
        # running_gym_sequential_vectorized.py:53-58
        term = self.terminated
        shifted = torch.cat([self.window[:, :, 1:], nxt[..., None]], dim=2)
        full = nxt[..., None].repeat(1, 1, self.W)
        self.window = torch.where(term[:, None, None], full, shifted)
        self.t += 1

    def get_state(self, normalize: bool):
        return get_state(self.window, normalize)

    # ---- the single evaluation env of Algorithm.test (base_algorithm.py:21-48): env 0 of the
    # streams, restarted at stream step 0 by every test reset --------------------------------
    def test_reset(self):
        """helper.py:59-67 with test_phase=True: window (1, O, W) := the reset observation."""
        self.test_t = 0
        self.test_window = self.base_obs[0, :1].double()[..., None].repeat(1, 1, self.W)

    def test_reset_window(self):
        """reset_environment(test_phase=True) after a termination (base_algorithm.py:33-34)."""
        self.test_reset()

    def test_env_step(self, action: torch.Tensor):
        """test_environment.step(action (A,)) -> (observation, reward, terminated, truncated,
        info) with the synthetic dynamics at stream step k."""
        k = self.test_t
        t_len = self.base_reward.shape[0]
        a = action.double()
        o = self.base_obs.shape[2]
        obs = self.base_obs[(k + 1) % (t_len + 1), 0].double() + 0.1 * a[torch.arange(o) % self.A]
        ctrl = 0.0
        for j in range(self.A):
            ctrl = ctrl + float(a[j]) * float(a[j])
        reward = float(self.base_reward[k % t_len, 0]) - 0.01 * ctrl
        terminated = bool(self.base_terminated[k % t_len, 0])
        self.test_t = k + 1
        return obs, reward, terminated, False, {}

    def test_get_state(self, normalize: bool):
        """running_gym_sequential_vectorized.py:83-92 with test_phase=True."""
        return get_state(self.test_window, normalize)


# ----------------------------------------------------------------------------------------------
# GAE (A7/A8) -- torchrl 0.6.0 restated
# ----------------------------------------------------------------------------------------------
def generalized_advantage_estimate(gamma, lmbda, state_value, next_state_value, reward, done,
                                   terminated=None):
    """torchrl.objectives.value.functional.generalized_advantage_estimate (torchrl 0.6.0), time_dim=-2.

    dtype walk (why the engine carries the recurrence in f64): ``gamma * not_terminated`` is an f32
    tensor, ``reward`` is f64 (numpy rewards) so ``delta`` is f64; ``prev_advantage`` is the f64 RHS
    of the chained assignment while ``advantage`` stores f32.
    """
    if terminated is None:
        terminated = done.clone()
    if not (next_state_value.shape == state_value.shape == reward.shape == done.shape ==
            terminated.shape):
        raise RuntimeError(SHAPE_ERR)
    dtype = next_state_value.dtype
    not_done = (~done).int()
    not_terminated = (~terminated).int()
    *batch_size, time_steps, lastdim = not_done.shape
    advantage = torch.empty(*batch_size, time_steps, lastdim, dtype=dtype)
    prev_advantage = 0
    g_not_terminated = gamma * not_terminated
    delta = reward + (g_not_terminated * next_state_value) - state_value
    discount = lmbda * gamma * not_done
    for t in reversed(range(time_steps)):
        prev_advantage = advantage[..., t, :] = delta[..., t, :] + (prev_advantage *
                                                                    discount[..., t, :])
    value_target = advantage + state_value
    return advantage, value_target


# ----------------------------------------------------------------------------------------------
# PPO loop (ppo.py:13-159)
# ----------------------------------------------------------------------------------------------
@torch.no_grad()
def rollout(env: RefSyntheticEnv, agent: RefAgent) -> Dict[str, torch.Tensor]:
    """ppo.py:13-60 -> the (N, T) buffer (TensorDict ``cat(dim=1)``) as a dict of tensors."""
    cfg = agent.cfg
    env.reset()
    next_state = env.get_state(cfg.normalize_observations)
    items: Dict[str, list] = {k: [] for k in (
        "current_state", "current_state_value", "next_state_value", "action", "action_log_prob",
        "reward", "terminated", "truncated")}
    for _ in range(cfg.horizon):
        current_state = torch.clone(next_state)
        current_state_value = agent.get_state_value(current_state)
        sub_actions, dist = agent.act(current_state, return_dist=True, test_phase=False)
        action_log_prob = dist.log_prob(sub_actions).sum(dim=1)
        env.step(sub_actions)
        next_state = env.get_state(cfg.normalize_observations)
        next_state_value = agent.get_state_value(next_state)
        items["current_state"].append(current_state.unsqueeze(1))
        items["current_state_value"].append(current_state_value.unsqueeze(1))
        items["next_state_value"].append(next_state_value.unsqueeze(1))
        items["action"].append(sub_actions.unsqueeze(1))
        items["action_log_prob"].append(action_log_prob.unsqueeze(1))
        items["reward"].append(env.reward.clone()[:, None].unsqueeze(1))
        items["terminated"].append(env.terminated.clone()[:, None])
        items["truncated"].append(env.truncated.clone()[:, None])
    return {k: torch.cat(v, dim=1) for k, v in items.items()}


@torch.no_grad()
def calculate_advantages(memory: Dict[str, torch.Tensor], cfg: RefConfig) -> None:
    """ppo.py:62-91 (adds ``advantage`` and ``current_state_value_target`` to ``memory``)."""
    rewards = memory["reward"]
    if cfg.normalize_rewards:
        rewards = rewards - rewards.mean(dim=1).unsqueeze(1)
        rewards = (rewards / rewards.std(dim=1).unsqueeze(1)) * cfg.advantage_scaler
    terminated = memory["terminated"].unsqueeze(-1)
    done = torch.clone(terminated)
    done[:, -1, :] = True
    advantage, value_target = generalized_advantage_estimate(
        cfg.gamma, cfg.lmbda, memory["current_state_value"], memory["next_state_value"], rewards,
        done, terminated)
    if cfg.normalize_advantage:
        advantage = advantage - advantage.mean(dim=1).unsqueeze(1)
        advantage = (advantage / advantage.std(dim=1).unsqueeze(1)) * cfg.advantage_scaler
        value_target = value_target - value_target.mean(dim=1).unsqueeze(1)
        value_target = (value_target / value_target.std(dim=1).unsqueeze(1)) * cfg.advantage_scaler
    memory["current_state_value_target"] = value_target
    memory["advantage"] = advantage


def train(agent: RefAgent, memory: Dict[str, torch.Tensor], current_episode: int = 0,
          max_minibatches: Optional[int] = None) -> Tuple[float, float]:
    """ppo.py:93-154.  ``max_minibatches`` stops early (tight single-minibatch parity tests)."""
    cfg = agent.cfg
    batch_size = cfg.batch_size
    epochs = cfg.epochs
    n_envs, horizon = memory["action"].shape[:2]
    batches_per_epoch = int(horizon * n_envs / batch_size)
    flat = {k: v.reshape(n_envs * horizon, *v.shape[2:]) for k, v in memory.items()}
    epoch_losses: List[List[float]] = [[], []]
    done_minibatches = 0
    for _ in range(epochs):
        iteration_losses: List[List[float]] = [[], []]
        idx = torch.randperm(n_envs * horizon)
        shuffled = {k: v[idx] for k, v in flat.items()}
        for i in range(batches_per_epoch):
            batch = {k: v[int(i * batch_size):int((i + 1) * batch_size)] for k, v in shuffled.items()}
            if len(batch["action"]) != batch_size:
                continue
            if max_minibatches is not None and done_minibatches >= max_minibatches:
                return float("nan"), float("nan")
            sub_actions = batch["action"]
            _, distributions = agent.act(batch["current_state"], return_dist=True)
            action_log_prob = batch["action_log_prob"]
            new_action_log_prob = distributions.log_prob(sub_actions).sum(dim=1)
            current_state_value = agent.get_state_value(batch["current_state"])
            critic_loss = huber_loss(current_state_value, batch["current_state_value_target"],
                                     reduction="mean")
            agent.optimizers["critic"].zero_grad()
            critic_loss.backward()
            agent.optimizers["critic"].step()
            advantage = batch["advantage"]
            total_entropy = distributions.entropy().mean()
            ratio = (new_action_log_prob - action_log_prob).exp()[:, None]
            surrogate1 = ratio * advantage
            surrogate2 = torch.clamp(ratio, 1.0 - cfg.clip_epsilon, 1.0 + cfg.clip_epsilon) * advantage
            actor_loss = -torch.min(surrogate1, surrogate2).mean() - total_entropy * cfg.entropy_eps
            agent.optimizers["actor"].zero_grad()
            actor_loss.backward()
            agent.optimizers["actor"].step()
            # ppo.py:136-137 runs after both steps: it only rescales grads that the next
            # zero_grad(set_to_none=True) discards, so it never changes a parameter.
            torch.nn.utils.clip_grad_norm_(agent.networks.parameters(), cfg.max_grad_norm)
            iteration_losses[0].append(actor_loss.detach().item())
            iteration_losses[1].append(critic_loss.detach().item())
            done_minibatches += 1
        if iteration_losses[0]:
            epoch_losses[0].append(sum(iteration_losses[0]) / len(iteration_losses[0]))
            epoch_losses[1].append(sum(iteration_losses[1]) / len(iteration_losses[1]))
        else:
            raise ZeroDivisionError("division by zero")  # ppo.py:142 on an empty epoch
    actor_loss_mean = sum(epoch_losses[0]) / len(epoch_losses[0])
    critic_loss_mean = sum(epoch_losses[1]) / len(epoch_losses[1])
    if current_episode < 2500:
        for scheduler in agent.schedulers.values():
            scheduler.step()
    return actor_loss_mean, critic_loss_mean


def iterate(env: RefSyntheticEnv, agent: RefAgent, current_episode: int = 0):
    """ppo.py:156-159 (PPO._iterate)."""
    memory = rollout(env, agent)
    calculate_advantages(memory, agent.cfg)
    losses = train(agent, memory, current_episode)
    return memory, losses


@torch.no_grad()
def test(env: RefSyntheticEnv, agent: RefAgent, steps: int = 1000) -> float:
    """base_algorithm.py:21-48 (Algorithm.test, visualize=False): deterministic mean-action
    rollout of the single test env, reset on termination, window shift + append otherwise."""
    cfg = agent.cfg
    rewards = []
    env.test_reset()
    next_state = env.test_get_state(cfg.normalize_observations)
    for _ in range(steps):
        current_state = torch.clone(next_state)
        action, _ = agent.act(current_state, return_dist=True, test_phase=True)
        last_observation, reward, terminated, _, _ = env.test_env_step(action.reshape(-1))
        if terminated:
            env.test_reset_window()
        else:
            # helper.py:51-57 (test_phase) then observation[:, -1] = last_observation
            env.test_window[..., :-1] = env.test_window[..., 1:].clone()
            env.test_window[0, :, -1] = last_observation
        rewards.append(reward)
        next_state = env.test_get_state(cfg.normalize_observations)
    return sum(rewards) / len(rewards)


def flat_params(agent: RefAgent) -> torch.Tensor:
    """All parameters, actor then critic, in state_dict order (the engine's flat layout)."""
    return torch.cat([p.detach().reshape(-1) for p in agent.networks.parameters()])


def adam_reference_step(p, g, m, v, step: int, lr: float, beta1=0.9, beta2=0.999, eps=1e-8):
    """One ``torch.optim.Adam`` single-tensor step (adam.py ``_single_tensor_adam``) on CPU
    tensors, in place, via the real optimizer -- the checker for the engine's fused Adam."""
    param = torch.nn.Parameter(p.clone())
    opt = torch.optim.Adam([param], lr=lr, betas=(beta1, beta2), eps=eps)
    st = opt.state[param]
    st["step"] = torch.tensor(float(step - 1))
    st["exp_avg"] = m.clone()
    st["exp_avg_sq"] = v.clone()
    param.grad = g.clone()
    opt.step()
    st = opt.state[param]
    return param.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone()


def math_log_sqrt_2pi() -> float:
    return math.log(math.sqrt(2 * math.pi))


# ---- bf16 GEMM emulation (engine precision "bf16"; not a reference behaviour) ----------------
# BASELINE.json configs[1] names "bf16 GEMMs with fp32 accumulate and fp32 master params": every
# fc layer of both nets -- the hidden layers AND the head (last_layer) -- multiplies bf16-rounded
# operands with f32 accumulation; biases, activations, the distribution / loss math, GAE and Adam
# stay f32.
def _bf(x: torch.Tensor) -> torch.Tensor:
    """Round to bf16 (round-to-nearest-even, as v_cvt_pk_bf16_f32) and back to x's dtype (f32;
    f64 for the f64-accumulated emulation the bf16 gradient tests compare against)."""
    return x.to(torch.bfloat16).to(x.dtype)


class _BF16Linear(torch.autograd.Function):
    """y = bf16(x) @ bf16(W)^T + b with f32 accumulation; backward GEMMs also on bf16-rounded
    operands (dx = bf16(dy) @ bf16(W), dW = bf16(dy)^T @ bf16(x)); db = sum dy in f32 (the
    engine sums the f32 dY before rounding) -- what the engine's bf16 MFMAs compute for every fc
    layer (gemm_bf16_kernel, the fused kernels' 32x32x16 / 16x16x32 products, and the VALU head
    kernels on rounded operands)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        y = _bf(x) @ _bf(w).t()
        return y + b if b is not None else y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        g = _bf(gy)
        return g @ _bf(w), g.t() @ _bf(x), (gy.sum(0) if ctx.has_b else None)


def use_bf16_gemms(agent: "RefAgent") -> None:
    """Switch every Linear layer of both nets (hidden layers and head) to the bf16-operand GEMM."""
    for net in (agent.networks["actor"].actor, agent.networks["critic"].network):
        for mod in list(net.first_layers) + [net.last_layer]:
            if isinstance(mod, nn.Linear):
                mod.forward = (lambda m: (lambda x: _BF16Linear.apply(x, m.weight, m.bias)))(mod)
