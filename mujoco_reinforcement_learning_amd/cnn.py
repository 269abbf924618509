"""Pixel-observation actor-critic (BASELINE.json configs[4]: dm_control cheetah-run, 84x84x3
frames, 1024 envs) on the MI355X engine.

The reference has no pixel / CNN path (``running_dm_control.py:56-91`` is a
state-observation humanoid, and no model takes images), so the encoder is this engine's
declaration, kept as close to the reference's model family as possible:

  * ``PixelEncoder``      the Nature-DQN stack Conv2d(3, 32, 8, 4) ReLU, Conv2d(32, 64, 4, 2)
                          ReLU, Conv2d(64, 64, 3, 1) ReLU, Flatten -> 3136 features, initialised
                          like the reference's hidden layers (network_block_creator.py:18-21:
                          orthogonal sqrt(2), zero bias, after the module's own default init);
  * ``EngineCNNActor``    encoder + the reference NetworkBlock actor head and state-independent
                          ``actor_logstd`` (models/linear/actor.py:9-30);
  * ``EngineCNNCritic``   encoder + NetworkBlock value head (models/critic.py:6-25);
  * ``CNNEngine``         the ``ppo_cnn_ctx`` front end (csrc/cnn_engine.hip, implicit-GEMM
                          convolutions on MFMA, csrc/conv.h) with the ``Engine`` methods the PPO
                          loop calls (``policy_step``, ``minibatch_grad``);
  * ``CNNEngineAgent``    the PPOAgent surface (act / get_state_value / optimizers / save / load);
  * ``PixelRolloutBuffer`` the rollout buffer with u8 frames as ``current_state``;
  * ``SyntheticPixelVecEnvHelper`` the synthetic pixel VecEnv (physics is out of scope).

Actor and critic keep separate encoders: they have separate Adam optimizers (ppo_agent.py:15-22)
and the critic steps before the actor's loss is back-propagated (ppo.py:120-135).
"""
from __future__ import annotations

import ctypes
from types import SimpleNamespace
from typing import Dict, Optional

import numpy as np
import torch
from torch import nn

from . import _lib
from ._lib import check, ptr
from .agent import _ACT_NAMES, ExponentialLRFacade, FlatAdam, PPOEngineAgent
from .buffer import RolloutBuffer
from .engine import _need, _stream
from .environments import Timestep, make_synthetic_streams
from .features import Run
from .models import _Block, move_to_flat

FRAME = (84, 84, 3)                      # H, W, C of a dm_control pixel observation
FRAME_BYTES = FRAME[0] * FRAME[1] * FRAME[2]
FEATURES = 7 * 7 * 64                    # the encoder's flattened output


class PixelEncoder(nn.Sequential):
    """Nature-DQN encoder (parameters only; the forward runs in csrc/conv.h)."""

    def __init__(self):
        layers = []
        for cin, cout, k, s in ((3, 32, 8, 4), (32, 64, 4, 2), (64, 64, 3, 1)):
            conv = nn.Conv2d(cin, cout, k, s)
            with torch.no_grad():  # network_block_creator.py:18-21 (layer_init)
                torch.nn.init.orthogonal_(conv.weight, np.sqrt(2))
                conv.bias.fill_(0)
            layers += [conv, nn.ReLU()]
        super().__init__(*layers, nn.Flatten())


class EngineCNNActor(nn.Module):
    def __init__(self, hidden, act_dim: int, act_cls, use_bias: bool, output_max_value: float,
                 last_layer_std: float = 0.01):
        super().__init__()
        self.encoder = PixelEncoder()
        self.actor = _Block(FEATURES, hidden, act_dim, act_cls, use_bias, last_layer_std)
        self.actor_logstd = nn.Parameter(torch.zeros(act_dim))
        self.output_max_value = output_max_value
        self._agent = None

    def forward(self, x):
        mean = self._agent._actor_mean(x)
        std = self.actor_logstd.detach().exp()
        return mean, torch.repeat_interleave(std[None, :], mean.shape[0], dim=0)


class EngineCNNCritic(nn.Module):
    def __init__(self, hidden, act_cls, last_layer_std: float = 0.01):
        super().__init__()
        self.encoder = PixelEncoder()
        self.network = _Block(FEATURES, hidden, 1, act_cls, True, last_layer_std)
        self._agent = None

    def forward(self, x):
        return self._agent.get_state_value(x)


class CNNEngine:
    """One ``ppo_cnn_ctx``: encoder + MLP shapes, workspace and split-K slabs."""

    fused = False  # the staged-record path of the MLP engine does not apply

    def __init__(self, act_dim: int, hidden, activation: str = "relu", use_bias: bool = True,
                 output_max_value: float = 1.0, max_rows: int = 4096,
                 device: Optional[torch.device] = None):
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        cfg = _lib.CnnCfg()
        cfg.height, cfg.width, cfg.channels = FRAME
        cfg.act_dim = act_dim
        cfg.activation = _lib.ACT_CODES[activation]
        cfg.use_bias = int(bool(use_bias))
        cfg.n_hidden = len(hidden)
        for i, h in enumerate(hidden):
            cfg.hidden[i] = int(h)
        cfg.output_max_value = float(output_max_value)
        cfg.max_rows = int(max_rows)
        self.cfg = cfg
        self.act_dim = act_dim
        self.in_dim = FRAME_BYTES
        self.max_rows = int(max_rows)
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self.lib.ppo_cnn_ctx_create(ctypes.byref(cfg), self.device.index or 0,
                                              ctypes.byref(handle)))
        self._ctx = handle
        total, n_actor = ctypes.c_int64(), ctypes.c_int64()
        n = self.lib.ppo_cnn_param_layout(self._ctx, None, 0, ctypes.byref(total),
                                          ctypes.byref(n_actor))
        check(min(n, 0))
        arr = (ctypes.c_int64 * n)()
        self.lib.ppo_cnn_param_layout(self._ctx, arr, n, None, None)
        self._offsets = list(arr)
        self.n_params, self.n_actor = int(total.value), int(n_actor.value)
        self.n_critic = self.n_params - self.n_actor
        self.precision = "f32"
        self._params = None

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and ctx.value:
            try:
                self.lib.ppo_cnn_ctx_destroy(ctx)
            except Exception:  # interpreter shutdown
                pass
            self._ctx = None

    def param_offsets(self) -> list:
        return list(self._offsets)

    def bind(self, flat_params: torch.Tensor) -> None:
        _need(flat_params, "flat_params", torch.float32, (self.n_params,), self.device)
        check(self.lib.ppo_cnn_bind_params(self._ctx, ptr(flat_params)))
        self._params = flat_params

    def loss_entropy_share(self, share: float) -> None:
        """Share of the entropy bonus in the LOGGED actor loss (ppo_cnn_loss_entropy_share)."""
        check(self.lib.ppo_cnn_loss_entropy_share(self._ctx, float(share)))

    def set_precision(self, precision: str) -> None:
        if precision not in _lib.PREC_CODES:
            raise ValueError(f"unknown precision {precision!r}; use one of {sorted(_lib.PREC_CODES)}")
        check(self.lib.ppo_cnn_set_precision(self._ctx, _lib.PREC_CODES[precision]))
        self.precision = precision

    def set_rng_counter(self, counter: Optional[torch.Tensor]) -> None:
        if counter is not None:
            _need(counter, "counter", torch.int64, (1,), self.device)
        check(self.lib.ppo_cnn_set_rng_counter(self._ctx, ptr(counter)))
        self._rng_counter = counter

    def pack_weights(self) -> None:
        """The conv weights are repacked inside every forward (ppo_cnn_*)."""

    def _frames(self, frames: torch.Tensor) -> int:
        n = frames.shape[0]
        _need(frames, "frames", torch.uint8, device=self.device)
        if frames.numel() != n * FRAME_BYTES:
            raise RuntimeError(f"frames hold {frames.numel() // max(n, 1)} bytes per row, "
                               f"expected {FRAME} = {FRAME_BYTES}")
        return n

    def forward(self, frames: torch.Tensor, mean=None, value=None, feat_actor=None,
                feat_critic=None) -> None:
        n = self._frames(frames)
        for name, t, k in (("mean", mean, self.act_dim), ("value", value, 1),
                           ("feat_actor", feat_actor, FEATURES),
                           ("feat_critic", feat_critic, FEATURES)):
            if t is not None:
                _need(t, name, torch.float32, device=self.device)
                if t.numel() != n * k:
                    raise RuntimeError(f"{name} has {t.numel()} elements, expected {n * k}")
        check(self.lib.ppo_cnn_forward(self._ctx, ptr(frames), n, ptr(mean), ptr(value),
                                       ptr(feat_actor), ptr(feat_critic), _stream(self.device)))

    def policy_step(self, state: torch.Tensor, eps: Optional[torch.Tensor] = None, seed: int = 0,
                    offset: int = 0, action=None, logp=None, value=None, mean=None) -> None:
        """ppo.py:22-26 for one rollout step on u8 frames (the ``Engine.policy_step`` contract)."""
        n = self._frames(state)
        if eps is not None:
            _need(eps, "eps", torch.float32, (n, self.act_dim), self.device)
        for name, t, k in (("action", action, self.act_dim), ("logp", logp, 1),
                           ("value", value, 1), ("mean", mean, self.act_dim)):
            if t is not None:
                _need(t, name, torch.float32, device=self.device)
                if t.numel() != n * k:
                    raise RuntimeError(f"{name} has {t.numel()} elements, expected {n * k}")
        check(self.lib.ppo_cnn_policy_step(self._ctx, ptr(state), n, ptr(eps), seed, offset,
                                           ptr(action), ptr(logp), ptr(value), ptr(mean),
                                           _stream(self.device)))

    def minibatch_grad(self, states, actions, old_logp, adv, vtarget, rows, b: int, grad, loss,
                       clip_lo: float, clip_hi: float, entropy_coef: float, inv_b: float,
                       inv_ba: float, count: Optional[torch.Tensor] = None) -> None:
        """ppo.py:108-135 for one minibatch (the ``Engine.minibatch_grad`` contract); ``states``
        are the rollout buffer's u8 frames."""
        if count is not None:
            raise NotImplementedError("the pixel agent runs the single-process / local-DP paths")
        _need(states, "states", torch.uint8, device=self.device)
        _need(rows, "rows", torch.int32, device=self.device)
        _need(grad, "grad", torch.float32, (self.n_params,), self.device)
        if loss is not None:
            _need(loss, "loss", torch.float32, device=self.device)
        check(self.lib.ppo_cnn_minibatch_grad(
            self._ctx, ptr(states), ptr(actions), ptr(old_logp), ptr(adv), ptr(vtarget),
            ptr(rows), int(b), ptr(grad), ptr(loss), clip_lo, clip_hi, entropy_coef, inv_b,
            inv_ba, _stream(self.device)))

    # ---- measurement (the Engine.timing* contract of bench.py) ----------------------------------
    def timing(self, enable: bool, capacity: int = 65536) -> None:
        check(self.lib.ppo_cnn_timing(self._ctx, int(enable), int(capacity)))

    def timing_kernels(self) -> dict:
        out = {}
        n_k = self.lib.ppo_cnn_timing_kernel(self._ctx, -1, None, None, None, None, None, None)
        check(min(n_k, 0))
        for i in range(n_k):
            name, cls = ctypes.c_char_p(), ctypes.c_int()
            ms, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
            cnt = ctypes.c_int64()
            check(self.lib.ppo_cnn_timing_kernel(self._ctx, i, ctypes.byref(name),
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


class PixelRolloutBuffer(RolloutBuffer):
    """RolloutBuffer (time-major, buffer.py) whose states are u8 frames (T+1, N, H*W*C);
    ``memory["current_state"]`` is the (N, T, H, W, C) view."""

    def __init__(self, num_envs: int, horizon: int, act_dim: int, device: torch.device):
        super().__init__(num_envs, horizon, 1, 1, act_dim, device)
        self.states = torch.empty(horizon + 1, num_envs, FRAME_BYTES, dtype=torch.uint8,
                                  device=device)

    def __getitem__(self, key: str) -> torch.Tensor:
        if key == "current_state":
            t = self.horizon
            return self.states[:t].view(t, self.num_envs, *FRAME).permute(1, 0, 2, 3, 4)
        return super().__getitem__(key)


class CNNEngineAgent(PPOEngineAgent):
    """PPOAgent (ppo_agent.py:10-43) with the pixel actor / critic on the engine."""

    def __init__(self, run: Optional[Run] = None, device: Optional[torch.device] = None,
                 max_rows: Optional[int] = None):
        run = run or Run.instance()
        if run is None:
            raise ValueError("CNNEngineAgent needs a Run (construct entities Run first)")
        self.run = run
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        nc, ec = run.network_config, run.environment_config
        act_cls = nc.activation_class
        if act_cls not in _ACT_NAMES:
            raise ValueError(f"activation {act_cls} not supported by the engine (ReLU/Tanh/ELU)")
        hidden = list(nc.linear_hidden_shapes)[:nc.num_linear_layers]
        # the pixel engine builds both heads with one width list; record it as the critic's so a
        # saved run (Run.save) describes the networks.pth it sits beside
        ch = run.engine_config.critic_hidden_shapes
        if ch is not None and list(ch) != hidden:
            raise ValueError(f"the CNN engine's critic head uses the actor's widths {hidden}, "
                             f"not critic_hidden_shapes={list(ch)}")
        run.engine_config.critic_hidden_shapes = list(hidden)
        self.networks = nn.ModuleDict()
        # PPOAgent.initialize_networks: Actor() then Critic() (RNG order)
        self.networks["actor"] = EngineCNNActor(hidden, nc.output_shape, act_cls, nc.use_bias,
                                                nc.output_max_value, nc.last_layer_std)
        self.networks["critic"] = EngineCNNCritic(hidden, act_cls, nc.last_layer_std)
        for m in (self.networks["actor"], self.networks["critic"]):
            m._agent = self
        rows = max_rows or max(ec.num_envs, int(run.training_config.batch_size))
        self.engine = CNNEngine(nc.output_shape, hidden, _ACT_NAMES[act_cls], nc.use_bias,
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

    def make_buffer(self, num_envs: int, horizon: int) -> PixelRolloutBuffer:
        return PixelRolloutBuffer(num_envs, horizon, self.engine.act_dim, self.device)

    def _as_state(self, state: torch.Tensor) -> torch.Tensor:
        if state.dtype != torch.uint8:
            raise ValueError(f"pixel states are u8 frames, got {state.dtype}")
        s = state.to(device=self.device)
        return s.reshape(len(s), -1).contiguous()


# ---- synthetic pixel VecEnv ------------------------------------------------------------------------
def synthetic_pixel_step(seed: int, t: int, action: Optional[torch.Tensor], frames_out: torch.Tensor,
                         base_reward=None, base_term=None, reward_out=None, term_out=None) -> None:
    """ppo_synthetic_pixel_step: frame t of every env (include/ppo_engine.h formula) into
    frames_out (N, H*W*C) u8; with the base streams also step t-1's reward / termination."""
    lib = _lib.load()
    n = frames_out.shape[0]
    dev = frames_out.device
    _need(frames_out, "frames_out", torch.uint8, device=dev)
    a = 0
    if action is not None:
        _need(action, "action", torch.float32, device=dev)
        a = action.shape[1]
    if reward_out is not None:
        _need(base_reward, "base_reward", torch.float32, device=dev)
        _need(base_term, "base_term", None, device=dev)
        _need(reward_out, "reward_out", torch.float64, (n,), dev)
        _need(term_out, "term_out", None, (n,), dev)
    check(lib.ppo_synthetic_pixel_step(int(seed) & 0xFFFFFFFF, int(t), ptr(action), n, FRAME[0],
                                       FRAME[1], FRAME[2], max(a, 1), ptr(frames_out),
                                       ptr(base_reward), ptr(base_term), ptr(reward_out),
                                       ptr(term_out), _stream(dev)))


class SyntheticPixelVecEnvHelper:
    """EnvironmentHelper (helper.py:12-67) over the synthetic pixel VecEnv: frames from
    ppo_synthetic_pixel_step (the next frame depends on the action, so the T rollout steps stay
    sequential), rewards / terminations from the same base streams and formulas as the state env
    (environments.SyntheticVecEnvHelper).  window_length is 1: the state is the current frame."""

    writes_into_buffer = True
    graph_safe = True

    def __init__(self, streams: Optional[dict] = None, run: Optional[Run] = None,
                 device: Optional[torch.device] = None, seed: int = 0, p_terminate: float = 0.0):
        self.rewards, self.memory, self.images = [], [], []
        self.run = run or Run.instance()
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self._streams = streams
        self.seed = int(seed)
        self._p_terminate = p_terminate
        self.initialize()

    def initialize(self):
        ec, nc = self.run.environment_config, self.run.network_config
        n, t = ec.num_envs, ec.maximum_timesteps
        self.num_envs, self.horizon, self.act_dim = n, t, nc.output_shape
        streams = self._streams or make_synthetic_streams(n, t, 1, self.seed, self._p_terminate)
        dev = self.device
        self.base_reward = streams["base_reward"].to(dev, torch.float32).contiguous()
        self.base_terminated = streams["base_terminated"].to(dev, torch.bool).contiguous()
        self._frame = torch.empty(n, FRAME_BYTES, dtype=torch.uint8, device=dev)
        self.timestep = Timestep(self._frame.view(n, *FRAME), torch.zeros(n, dtype=torch.float64,
                                                                          device=dev),
                                 torch.zeros(n, dtype=torch.bool, device=dev),
                                 torch.zeros(n, dtype=torch.bool, device=dev), {})
        self.environment = SimpleNamespace(num_envs=n, timestep=self.timestep)
        self.test_environment = SimpleNamespace(num_envs=1)
        self.t = 0

    def reset(self, release_memory: bool = True):
        self.rewards, self.images = [], []
        if release_memory:
            self.memory = []

    def reset_environment(self, test_phase: bool):
        if test_phase:
            raise NotImplementedError("the synthetic pixel helper has no evaluation env")
        self.t = 0
        synthetic_pixel_step(self.seed, 0, None, self._frame)
        self.timestep.terminated.zero_()
        self.timestep.truncated.zero_()

    def step(self, action: torch.Tensor, reward_out: Optional[torch.Tensor] = None,
             terminated_out: Optional[torch.Tensor] = None):
        t = self.t
        if t >= self.horizon:
            raise RuntimeError("synthetic pixel VecEnv: horizon exhausted; call reset_environment()")
        reward = reward_out if reward_out is not None else self.timestep.reward
        term = terminated_out if terminated_out is not None else self.timestep.terminated
        synthetic_pixel_step(self.seed, t + 1, action.contiguous(), self._frame, self.base_reward,
                             self.base_terminated, reward, term)
        self.timestep.reward = reward
        self.timestep.terminated = term
        self.t = t + 1

    def get_state(self, test_phase: bool = False, out: Optional[torch.Tensor] = None):
        """(N, H, W, C) u8 frames (the pixel analogue of get_state's (N, W, O))."""
        if test_phase:
            raise NotImplementedError("the synthetic pixel helper has no evaluation env")
        n = self.num_envs
        if out is None:
            return self._frame.clone().view(n, *FRAME)
        out.view(n, FRAME_BYTES).copy_(self._frame)
        return out.view(n, *FRAME)
