"""CPU oracle for the windowed BiLSTM actor-critic.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, as the checker; the product package never imports
it and has no fallback to it.

What it restates (reference = aminrezaee/mujoco_reinforcement_learning @ 2025-03-03):

* ``bilstm``            torch.nn.LSTM(input, hidden, num_layers, bidirectional=True,
                        batch_first=True) as LSTMActor / LSTMCritic build it
                        (models/lstm/lstm_actor.py:12-16, lstm_critic.py:19-23), written out
                        cell by cell in torch's CPU formulation: the input projection of every
                        step first, then per step gates = (h W_hh^T + b_hh) + (x W_ih^T + b_ih),
                        i, f, o = sigmoid, g = tanh, c = f*c + i*g, h = o*tanh(c); the reverse
                        direction runs t = W-1..0; a layer's output is [h_fwd, h_rev]
* ``RefLSTMActor``      lstm_actor.py:41-48: act() on the outputs flattened to (B, W*2L),
                        mean = tanh(MLP(.)), std = 0.2 * exp(tanh(MLP_logstd(.))) -- returned per
                        row as (B, A) (the reference's repeat_interleave at :48 makes it (B, B, A);
                        its row 0 is this std)
* ``RefLSTMCritic``     lstm_critic.py:33-41: value = MLP(act(Y[:, -1, :]))
* ``RefLSTMAgent``      ppo_agent.py:10-43 with those two networks; ``ppo_ref.rollout`` /
                        ``train`` drive it unchanged (ppo.py:13-154)

Parity pinning: tests/golden/gen_golden_lstm.py imports the reference's own LSTMActor /
LSTMCritic from /root/reference/src and records their init digests, forward outputs and the
gradients of the PPO minibatch losses (ppo.py:108-135 with the per-row std) into
tests/golden/reference_lstm.npz; tests/test_oracle.py checks this restatement against them.
"""
from __future__ import annotations

from typing import List, Sequence

import torch
from torch import nn

from .ppo_ref import ACTIVATIONS, MLPBlock, RefConfig, _BF16Linear, _bf, use_bf16_gemms as _mlp_bf16


class _BF16GateLinear(_BF16Linear):
    """_BF16Linear for the BiLSTM's gate products (X W_ih^T + b_ih, h W_hh^T + b_hh): the same
    bf16-operand GEMMs, but the bias gradient is the sum of the bf16-ROUNDED gate gradient dG --
    what csrc/bilstm.hip computes in bf16 mode, where the cell backward writes dG once as bf16 and
    both the weight-gradient GEMMs and the b_ih / b_hh column sums (gemm_bf16_kernel's COLSUM,
    wide_gemm.h's acol) read that one bf16 copy."""

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        g = _bf(gy)
        return g @ _bf(w), g.t() @ _bf(x), (g.sum(0) if ctx.has_b else None)


def _linear(x, w, b, bf16: bool):
    """torch's F.linear, or the bf16-operand product of the engine's PPO_PREC_BF16 mode
    (_BF16GateLinear: both operands rounded to bf16, accumulation in x's dtype, f32 bias, the bias
    gradient summed from bf16(dG)) -- not a reference behaviour."""
    if not bf16:
        return torch.nn.functional.linear(x, w, b)
    lead = x.shape[:-1]
    return _BF16GateLinear.apply(x.reshape(-1, x.shape[-1]), w, b).reshape(*lead, w.shape[0])


def lstm_direction(x: torch.Tensor, w_ih, w_hh, b_ih, b_hh, reverse: bool,
                   bf16: bool = False) -> torch.Tensor:
    """One direction of one layer over x (B, W, I) -> h (B, W, L) (torch CPU LSTM cell order).
    bf16=True: every GEMM of the layer (input projection, per-step recurrent projection, and so
    their backward dgrad / wgrad) on bf16-rounded operands; the cells stay in x's dtype."""
    b, w, _ = x.shape
    hidden = w_hh.shape[1]
    gx = _linear(x, w_ih, b_ih, bf16)  # every step's input projection at once
    h = x.new_zeros(b, hidden)
    c = x.new_zeros(b, hidden)
    out: List[torch.Tensor] = [None] * w
    steps = range(w - 1, -1, -1) if reverse else range(w)
    for t in steps:
        gates = _linear(h, w_hh, b_hh, bf16) + gx[:, t]
        i, f, g, o = gates.chunk(4, 1)
        i, f, g, o = i.sigmoid(), f.sigmoid(), g.tanh(), o.sigmoid()
        c = f * c + i * g
        h = o * c.tanh()
        out[t] = h
    return torch.stack(out, dim=1)


def bilstm(x: torch.Tensor, lstm: nn.LSTM) -> torch.Tensor:
    """Multi-layer bidirectional LSTM over x (B, W, I) with ``lstm``'s parameters -> (B, W, 2L)."""
    y = x
    bf16 = bool(getattr(lstm, "_ppo_bf16", False))  # set by use_bf16_gemms
    for layer in range(lstm.num_layers):
        outs = []
        for rev, sfx in ((False, ""), (True, "_reverse")):
            p = [getattr(lstm, f"{n}_l{layer}{sfx}") for n in ("weight_ih", "weight_hh", "bias_ih",
                                                                "bias_hh")]
            outs.append(lstm_direction(y, *p, reverse=rev, bf16=bf16))
        y = torch.cat(outs, dim=2)
    return y


class RefLSTMActor(nn.Module):
    """models/lstm/lstm_actor.py:9-48 (init in the reference's RNG order)."""

    def __init__(self, cfg: RefConfig, latent: int, layers: int, last_layer_std: float = 0.01):
        super().__init__()
        self.cfg = cfg
        self.feature_extractor = nn.LSTM(cfg.obs_dim, latent, num_layers=layers,
                                         bidirectional=True, batch_first=True)
        in_dim = latent * 2 * cfg.window
        act = ACTIVATIONS[cfg.activation]
        self.actor = MLPBlock(in_dim, cfg.actor_hidden, cfg.act_dim, act, nn.Tanh, cfg.use_bias,
                              last_layer_std)
        self.actor_logstd = MLPBlock(in_dim, cfg.actor_hidden, cfg.act_dim, act, nn.Tanh,
                                     cfg.use_bias, last_layer_std)

    def lstm_out(self, x):
        return bilstm(x.reshape(len(x), self.cfg.window, self.cfg.obs_dim), self.feature_extractor)

    def forward(self, x):
        features = ACTIVATIONS[self.cfg.activation]()(self.lstm_out(x).reshape(len(x), -1))
        mean = self.actor(features)
        std = 0.2 * self.actor_logstd(features).exp()
        return mean, std


class RefLSTMCritic(nn.Module):
    """models/lstm/lstm_critic.py:9-41 (one BiLSTM layer, the last step's features)."""

    def __init__(self, cfg: RefConfig, latent: int, last_layer_std: float = 0.01):
        super().__init__()
        self.cfg = cfg
        self.feature_extractor = nn.Sequential(
            nn.LSTM(cfg.obs_dim, latent, bidirectional=True, batch_first=True))
        self.network = MLPBlock(latent * 2, cfg.actor_hidden, 1, ACTIVATIONS[cfg.activation], None,
                                cfg.use_bias, last_layer_std)

    def lstm_out(self, x):
        return bilstm(x.reshape(len(x), self.cfg.window, self.cfg.obs_dim),
                      self.feature_extractor[0])

    def forward(self, x):
        feats = ACTIVATIONS[self.cfg.activation]()(self.lstm_out(x)[:, -1, :])
        return self.network(feats)


class RefLSTMAgent:
    """PPOAgent (ppo_agent.py:10-43) with LSTMActor / LSTMCritic; the ``RefAgent`` interface."""

    def __init__(self, cfg: RefConfig, latent: int = 256, layers: int = 1,
                 last_layer_std: float = 0.01):
        self.cfg = cfg
        self.networks = nn.ModuleDict()
        self.networks["actor"] = RefLSTMActor(cfg, latent, layers, last_layer_std)
        self.networks["critic"] = RefLSTMCritic(cfg, latent, last_layer_std)
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


def ppo_minibatch_losses(agent, states, actions, old_logp, adv, vt, clip_epsilon: float,
                         entropy_eps: float):
    """ppo.py:108-133 for one minibatch (no optimizer step): (actor_loss, critic_loss)."""
    _, dist = agent.act(states, return_dist=True)
    new_logp = dist.log_prob(actions).sum(dim=1)
    value = agent.get_state_value(states)
    critic_loss = torch.nn.functional.huber_loss(value, vt, reduction="mean")
    entropy = dist.entropy().mean()
    ratio = (new_logp - old_logp).exp()[:, None]
    s1 = ratio * adv
    s2 = torch.clamp(ratio, 1.0 - clip_epsilon, 1.0 + clip_epsilon) * adv
    actor_loss = -torch.min(s1, s2).mean() - entropy * entropy_eps
    return actor_loss, critic_loss


def minibatch_grads(agent, states, actions, old_logp, adv, vt, clip_epsilon: float,
                    entropy_eps: float):
    """Gradients of both losses w.r.t. every parameter, actor then critic, flattened in
    parameters() order, plus the two loss values."""
    for p in agent.networks.parameters():
        p.grad = None
    actor_loss, critic_loss = ppo_minibatch_losses(agent, states, actions, old_logp, adv, vt,
                                                   clip_epsilon, entropy_eps)
    (actor_loss + critic_loss).backward()  # disjoint parameter sets: each loss its own net
    g = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                   for p in agent.networks.parameters()])
    return g, float(actor_loss.detach()), float(critic_loss.detach())


def param_names(agent) -> Sequence[str]:
    return [f"{k}.{n}" for k in ("actor", "critic") for n, _ in agent.networks[k].named_parameters()]


# ---- bf16 GEMM emulation of the BiLSTM agent (engine precision "bf16"; not a reference behaviour)
def use_bf16_gemms(agent: RefLSTMAgent) -> None:
    """Switch every product of both nets to the engine's PPO_PREC_BF16 arithmetic
    (csrc/bilstm.hip: every GEMM rounds both operands to bf16, RNE, and accumulates in f32; bias
    adds, the LSTM cells, activations, the distribution and the losses stay f32):
      * the BiLSTMs (lstm_actor.py:12-16, lstm_critic.py:19-23): the input projection X W_ih^T, the
        per-step recurrent projection h W_hh^T, and through autograd their backward products
        (dG W_hh, dG W_ih, dG^T X, dG^T h_prev) on bf16(dG); the b_ih / b_hh gradients summed
        from the same bf16(dG) (_BF16GateLinear), as the engine sums them;
      * the MLP heads (NetworkBlock, lstm_actor.py:17-38, lstm_critic.py:24-31): ppo_ref's
        _BF16Linear on every Linear.
    Run it on an agent cast to float64 (``agent.networks.double()`` with f64 inputs) for the
    f64-accumulated emulation the bf16 kernels are held to: the same bf16-rounded operands, sums
    without f32 rounding."""
    nets = agent.networks
    for lstm in (nets["actor"].feature_extractor, nets["critic"].feature_extractor[0]):
        lstm._ppo_bf16 = True
    blocks = (nets["actor"].actor, nets["actor"].actor_logstd, nets["critic"].network)
    for blk in blocks:
        for mod in list(blk.first_layers) + [blk.last_layer]:
            if isinstance(mod, nn.Linear):
                mod.forward = (lambda m: (lambda x: _BF16Linear.apply(x, m.weight, m.bias)))(mod)
