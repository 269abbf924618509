"""Device rollout buffer with the reference TensorDict key/shape contract (ppo.py:30-50, :60, :90-91).

Storage is TIME-major in HBM (element (n, t) at row t*N + n) -- one rollout step writes one
contiguous block, the GAE/normalisation scans read coalesced rows, and ``current_state_value`` /
``next_state_value`` are two offset views of one (T+1, N) value array (V'_t = V_{t+1}: the reference
evaluates the critic twice on the identical tensor, ppo.py:22,29).  ``memory[key]`` returns the
reference's env-major (N, T, ...) shape as a zero-copy permuted view.
"""
from __future__ import annotations

import torch

KEYS = ("current_state", "current_state_value", "next_state_value", "action", "action_log_prob",
        "reward", "terminated", "truncated", "advantage", "current_state_value_target")


class RolloutBuffer:
    def __init__(self, num_envs: int, horizon: int, obs_dim: int, window: int, act_dim: int,
                 device: torch.device, reward_dtype=torch.float64):
        n, t = num_envs, horizon
        self.num_envs, self.horizon = n, t
        self.obs_dim, self.window, self.act_dim = obs_dim, window, act_dim
        self.device = device
        f32 = dict(dtype=torch.float32, device=device)
        self.states = torch.empty(t + 1, n, window * obs_dim, **f32)   # slot T holds s_T
        self.values = torch.empty(t + 1, n, **f32)
        self.actions = torch.empty(t, n, act_dim, **f32)
        self.logp = torch.empty(t, n, **f32)
        self.reward = torch.empty(t, n, dtype=reward_dtype, device=device)
        self.terminated = torch.zeros(t, n, dtype=torch.bool, device=device)
        self.truncated = torch.zeros(t, n, dtype=torch.bool, device=device)
        self.advantage = torch.empty(t, n, **f32)
        self.value_target = torch.empty(t, n, **f32)
        self.reward_work = None  # scratch for normalize_rewards (the reference keeps memory['reward'])

    # ---- TensorDict-like access (env-major views) -------------------------------------------
    def __getitem__(self, key: str) -> torch.Tensor:
        t = self.horizon
        if key == "current_state":
            return self.states[:t].view(t, self.num_envs, self.window,
                                        self.obs_dim).permute(1, 0, 2, 3)
        if key == "current_state_value":
            return self.values[:t].t().unsqueeze(-1)
        if key == "next_state_value":
            return self.values[1:].t().unsqueeze(-1)
        if key == "action":
            return self.actions.permute(1, 0, 2)
        if key == "action_log_prob":
            return self.logp.t()
        if key == "reward":
            return self.reward.t().unsqueeze(-1)
        if key == "terminated":
            return self.terminated.t()
        if key == "truncated":
            return self.truncated.t()
        if key == "advantage":
            return self.advantage.t().unsqueeze(-1)
        if key == "current_state_value_target":
            return self.value_target.t().unsqueeze(-1)
        raise KeyError(key)

    def __setitem__(self, key: str, value: torch.Tensor) -> None:
        """Write an env-major (N, T[, 1]) tensor into storage (ppo.py:90-91 semantics)."""
        dst = {"advantage": self.advantage, "current_state_value_target": self.value_target}.get(key)
        if dst is None:
            raise KeyError(f"{key} is not writable")
        v = value.reshape(self.num_envs, self.horizon).t()
        dst.copy_(v)

    def keys(self):
        return KEYS

    @property
    def batch_size(self):
        return torch.Size([self.num_envs, self.horizon])

    def __len__(self):
        return self.num_envs
