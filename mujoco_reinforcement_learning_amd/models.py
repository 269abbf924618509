"""Actor / critic modules whose parameters live in ONE flat fp32 device buffer.

The modules keep the reference's structure and state_dict keys so checkpoints interoperate
(SURVEY.md s8(f) rank 2):
  actor  -> ``actor_logstd``, ``actor.first_layers.{2i}.weight|bias``, ``actor.last_layer.*``
            (models/linear/actor.py:9-23 + network_block_creator.py:46-65)
  critic -> ``network.first_layers.{2i}.weight|bias``, ``network.last_layer.*``
            (models/critic.py:13-20, window flattened)
Initialisation replays the reference RNG order on the CPU (Linear default init, then
``orthogonal_(sqrt 2)`` + zero bias for hidden layers, ``orthogonal_(0.01)`` on the last weight,
network_block_creator.py:18-21,46-65), so a seeded engine starts from the reference's exact
parameters; the values are then moved into the flat buffer and every ``nn.Parameter`` becomes a
view of it.  Forward passes go through the engine's HIP kernels, never through torch ops.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch
from torch import nn


class _Block(nn.Module):
    """Parameter skeleton of ``NetworkBlock`` (no forward of its own)."""

    def __init__(self, in_dim: int, hidden: Sequence[int], out_dim: int, act_cls, use_bias: bool,
                 last_layer_std: float = 0.01):
        super().__init__()
        layers: List[nn.Module] = []
        width = in_dim
        for h in hidden:
            lin = nn.Linear(width, int(h), bias=use_bias)
            with torch.no_grad():
                torch.nn.init.orthogonal_(lin.weight, np.sqrt(2))
                if use_bias:
                    lin.bias.fill_(0)
            layers += [lin, act_cls()]
            width = int(h)
        self.first_layers = nn.Sequential(*layers)
        self.last_layer = nn.Linear(width, out_dim, bias=use_bias)
        with torch.no_grad():
            torch.nn.init.orthogonal_(self.last_layer.weight, last_layer_std)


class EngineActor(nn.Module):
    """models/linear/actor.py with the forward routed to the engine."""

    def __init__(self, in_dim: int, hidden, act_dim: int, act_cls, use_bias: bool,
                 output_max_value: float):
        super().__init__()
        self.actor = _Block(in_dim, hidden, act_dim, act_cls, use_bias)
        self.actor_logstd = nn.Parameter(torch.zeros(act_dim))
        self.output_max_value = output_max_value
        self._agent = None

    def forward(self, x):
        mean = self._agent._actor_mean(x)
        std = self.actor_logstd.detach().exp()
        return mean, torch.repeat_interleave(std[None, :], mean.shape[0], dim=0)


class EngineCritic(nn.Module):
    """models/critic.py (window flattened) with the forward routed to the engine."""

    def __init__(self, in_dim: int, hidden, act_cls):
        super().__init__()
        self.network = _Block(in_dim, hidden, 1, act_cls, True)
        self._agent = None

    def forward(self, x):
        return self._agent.get_state_value(x)


def move_to_flat(networks: nn.ModuleDict, device: torch.device, offsets: Sequence[int],
                 total: int) -> torch.Tensor:
    """Copy every parameter (``parameters()`` order: actor then critic) into one zero-padded
    flat device tensor at the engine's offsets (ppo_param_offsets: 16-float aligned) and
    re-point each ``nn.Parameter`` at its slice.  Returns the flat tensor."""
    slots = []
    for mod in networks.modules():
        for name, p in list(mod.named_parameters(recurse=False)):
            slots.append((mod, name, p))
    # networks.modules() visits parents before children but ``parameters()`` order is what the
    # C layout follows; rebuild the order from parameters() identity.
    order = {id(p): i for i, p in enumerate(networks.parameters())}
    slots.sort(key=lambda s: order[id(s[2])])
    if len(offsets) != len(slots):
        raise RuntimeError(f"engine layout has {len(offsets)} tensors, modules {len(slots)}")
    flat = torch.zeros(total, dtype=torch.float32, device=device)
    for (mod, name, p), off in zip(slots, offsets):
        n = p.numel()
        view = flat[off:off + n].view(p.shape)
        view.copy_(p.detach().to(torch.float32))
        setattr(mod, name, nn.Parameter(view, requires_grad=False))
    return flat
