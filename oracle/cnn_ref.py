"""CPU oracle for the pixel-observation actor-critic (BASELINE.json configs[4]).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / the timed CPU baseline.

**Parity unpinned by the reference.**  The reference has no pixel / CNN path
(running_dm_control.py:56-91 is a state-observation humanoid-run; no model takes images), so this
restates the engine's own declared model with plain torch-CPU modules:

* ``RefCNNActor``   Conv2d(3, 32, 8, 4) ReLU Conv2d(32, 64, 4, 2) ReLU Conv2d(64, 64, 3, 1) ReLU
                    Flatten (torch CHW order) -> the reference NetworkBlock actor head with tanh,
                    x output_max_value, and the state-independent ``actor_logstd``
                    (models/linear/actor.py:9-30; network_block_creator.py:18-86 via
                    ppo_ref.MLPBlock).  Pixels are u8 HWC frames scaled by x / 255.
* ``RefCNNCritic``  its own encoder + the NetworkBlock value head (models/critic.py:6-25).
* ``RefCNNAgent``   PPOAgent (ppo_agent.py:10-43): actor then critic, two Adams, two ExponentialLR.
* ``synthetic_frames`` / ``RefPixelEnv``  the synthetic pixel VecEnv of ppo_synthetic_pixel_step
                    (include/ppo_engine.h), restated in numpy integer arithmetic.

The PPO loop itself (rollout, GAE, train) is ppo_ref's restatement of ppo.py:13-159, driven with
these modules; ``use_bf16`` rounds every conv / linear operand to bf16 (f32 accumulate), the
engine's precision "bf16".
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from oracle import ppo_ref as R

FRAME = (84, 84, 3)


# ---- synthetic pixel VecEnv ------------------------------------------------------------------------
def _mix32(seed: int, t: int, n: np.ndarray, i: np.ndarray) -> np.ndarray:
    """mix32 of cnn_engine.hip in uint32 arithmetic (wrap-around multiplication)."""
    u = np.uint32
    with np.errstate(over="ignore"):
        h = (i.astype(u) * u(0x9E3779B1)) ^ (u(t * 0x85EBCA77 & 0xFFFFFFFF) +
                                             n.astype(u) * u(0xC2B2AE3D) +
                                             u(seed * 0x27D4EB2F & 0xFFFFFFFF))
        h ^= h >> u(16)
        h *= u(0x85EBCA6B)
        h ^= h >> u(13)
        h *= u(0xC2B2AE35)
        h ^= h >> u(16)
    return h


def synthetic_frames(seed: int, t: int, num_envs: int,
                     action: Optional[np.ndarray] = None) -> np.ndarray:
    """Frame t of every env, (N, H, W, C) u8:
    pix = (mix32(seed, t, n, (y*W + x)*C + c) + q[(2c + ((x + y) & 1)) % A]) & 255,
    q = clamp(floor(8 * action), -64, 63) (0 for the reset frame)."""
    h, w, c = FRAME
    n = np.arange(num_envs)[:, None]
    i = np.arange(h * w * c)[None, :]
    hsh = _mix32(seed, t, n, i).astype(np.int64)
    if action is None:
        q = np.zeros((num_envs, 1), dtype=np.int64)
        sel = np.zeros(h * w * c, dtype=np.int64)
    else:
        a = np.asarray(action, dtype=np.float32)
        q = np.clip(np.floor(a * np.float32(8.0)), -64, 63).astype(np.int64)
        ch = np.arange(h * w * c) % c
        pix = np.arange(h * w * c) // c
        x, y = pix % w, pix // w
        sel = (2 * ch + ((x + y) & 1)) % a.shape[1]
    return ((hsh + q[:, sel]) & 255).astype(np.uint8).reshape(num_envs, h, w, c)


class RefPixelEnv:
    """ppo_ref.RefSyntheticEnv's interface over pixel frames: step t -> t+1 draws frame t+1 from
    the action; reward = base_reward[t] - 0.01 * sum_a a^2 (f64, sequential in a); terminated =
    base_terminated[t].  get_state returns the (N, H, W, C) u8 frame (window_length 1)."""

    def __init__(self, seed: int, base_reward: torch.Tensor, base_terminated: torch.Tensor,
                 act_dim: int):
        self.seed = seed
        self.base_reward = base_reward
        self.base_terminated = base_terminated
        self.A = act_dim
        self.t = 0
        self.frame = None

    def reset(self):
        self.t = 0
        n = self.base_reward.shape[1]
        self.frame = torch.from_numpy(synthetic_frames(self.seed, 0, n))
        self.terminated = torch.zeros(n, dtype=torch.bool)
        self.truncated = torch.zeros(n, dtype=torch.bool)

    def step(self, action: torch.Tensor):
        t = self.t
        n = self.base_reward.shape[1]
        self.frame = torch.from_numpy(synthetic_frames(self.seed, t + 1, n, action.numpy()))
        a = action.double()
        ctrl = torch.zeros(n, dtype=torch.float64)
        for j in range(self.A):
            ctrl = ctrl + a[:, j] * a[:, j]
        self.reward = self.base_reward[t].double() - 0.01 * ctrl
        self.terminated = self.base_terminated[t].clone()
        self.truncated = torch.zeros(n, dtype=torch.bool)
        self.t += 1

    def get_state(self, normalize: bool):
        return self.frame.clone()


# ---- models --------------------------------------------------------------------------------------
def make_encoder() -> nn.Sequential:
    """Each Conv2d draws its default init, then orthogonal_(sqrt 2) and a zero bias -- the
    reference's layer_init (network_block_creator.py:18-21) applied to the encoder."""
    layers = []
    for cin, cout, k, s in ((3, 32, 8, 4), (32, 64, 4, 2), (64, 64, 3, 1)):
        conv = nn.Conv2d(cin, cout, k, s)
        with torch.no_grad():
            torch.nn.init.orthogonal_(conv.weight, np.sqrt(2))
            conv.bias.fill_(0)
        layers += [conv, nn.ReLU()]
    return nn.Sequential(*layers, nn.Flatten())


def _pixels(x: torch.Tensor) -> torch.Tensor:
    """(N, H, W, C) u8 -> (N, C, H, W) f32 in [0, 1] (x / 255)."""
    return (x.float() / 255.0).permute(0, 3, 1, 2)


class RefCNNActor(nn.Module):
    def __init__(self, cfg: R.RefConfig):
        super().__init__()
        self.cfg = cfg
        self.encoder = make_encoder()
        self.actor = R.MLPBlock(3136, cfg.actor_hidden, cfg.act_dim, R.ACTIVATIONS[cfg.activation],
                                nn.Tanh, cfg.use_bias)
        self.actor_logstd = nn.Parameter(torch.zeros(cfg.act_dim))

    def forward(self, x):
        mean = self.cfg.output_max_value * self.actor(self.encoder(_pixels(x)))
        std = self.actor_logstd[:self.cfg.act_dim].exp()
        return mean, torch.repeat_interleave(std[None, :], x.shape[0], dim=0)


class RefCNNCritic(nn.Module):
    def __init__(self, cfg: R.RefConfig):
        super().__init__()
        self.encoder = make_encoder()
        self.network = R.MLPBlock(3136, cfg.critic_hidden, 1, R.ACTIVATIONS[cfg.activation], None,
                                  True)

    def forward(self, x):
        return self.network(self.encoder(_pixels(x)))


class RefCNNAgent(R.RefAgent):
    """PPOAgent (ppo_agent.py:10-43) with the pixel actor / critic."""

    def __init__(self, cfg: R.RefConfig):
        self.cfg = cfg
        self.networks = nn.ModuleDict()
        self.networks["actor"] = RefCNNActor(cfg)
        self.networks["critic"] = RefCNNCritic(cfg)
        self.optimizers = {k: torch.optim.Adam(self.networks[k].parameters(), lr=cfg.learning_rate)
                           for k in ("actor", "critic")}
        self.schedulers = {k: torch.optim.lr_scheduler.ExponentialLR(self.optimizers[k], 0.999)
                           for k in ("actor", "critic")}


# ---- bf16 operand emulation (engine precision "bf16") ------------------------------------------
class _BF16Conv(torch.autograd.Function):
    """y = conv(bf16(x), bf16(W)) + b with f32 accumulation; dx = conv_transpose(bf16(dy),
    bf16(W)), dW = conv_wgrad(bf16(dy), bf16(x)), db = sum dy in f32 -- what conv.h's bf16
    products compute."""

    @staticmethod
    def forward(ctx, x, w, b, stride):
        ctx.save_for_backward(x, w)
        ctx.stride = stride
        return F.conv2d(R._bf(x), R._bf(w), b, stride)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        g = R._bf(gy)
        gx = torch.nn.grad.conv2d_input(x.shape, R._bf(w), g, ctx.stride)
        gw = torch.nn.grad.conv2d_weight(R._bf(x), w.shape, g, ctx.stride)
        return gx, gw, gy.sum((0, 2, 3)), None


def use_bf16(agent: RefCNNAgent) -> None:
    """Every conv and Linear operand of both nets rounded to bf16 (f32 accumulate)."""
    for net in (agent.networks["actor"], agent.networks["critic"]):
        for mod in net.encoder:
            if isinstance(mod, nn.Conv2d):
                mod.forward = (lambda m: (lambda x: _BF16Conv.apply(x, m.weight, m.bias,
                                                                    m.stride)))(mod)
        blk = net.actor if hasattr(net, "actor") else net.network
        for mod in list(blk.first_layers) + [blk.last_layer]:
            if isinstance(mod, nn.Linear):
                mod.forward = (lambda m: (lambda x: R._BF16Linear.apply(x, m.weight, m.bias)))(mod)


def features(agent: RefCNNAgent, frames: torch.Tensor):
    """The two encoders' flattened outputs (N, 3136) on u8 frames."""
    x = _pixels(frames)
    return agent.networks["actor"].encoder(x), agent.networks["critic"].encoder(x)
