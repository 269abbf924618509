"""VecEnv side of the drop-in: the ``EnvironmentHelper`` surface (helper.py:12-67,
running_gym_sequential_vectorized.py:19-100) over device-resident state.

``SyntheticVecEnvHelper`` is the benchmark / test environment.  MuJoCo physics is outside the hot
path; the harness drives the loop with synthetic dynamics whose next observation
depends on the action (so the T rollout steps stay sequential):

    obs'      = base_obs[t+1] + 0.1 * a[:, o % A]            (f64)
    reward    = base_reward[t] - 0.01 * sum_a a^2            (f64, a summed in order)
    terminated = base_terminated[t]

The observation window (N, O, W) f64 and its per-sample standardisation are the reference's
(``timestep.observation`` + ``get_state``), computed by the engine's A1 kernels.
"""
from __future__ import annotations

import ctypes

from dataclasses import dataclass, field
from types import SimpleNamespace
from typing import Optional

import torch

from . import engine as E
from .features import Run


@dataclass
class Timestep:
    """entities/timestep.py:5-11 with device tensors."""
    observation: torch.Tensor
    reward: torch.Tensor
    terminated: torch.Tensor
    truncated: torch.Tensor
    info: dict = field(default_factory=dict)


def make_synthetic_streams(num_envs: int, horizon: int, obs_dim: int, seed: int = 0,
                           p_terminate: float = 0.0, device=None) -> dict:
    """Seeded base streams: obs ~ N(0,1) (T+1, N, O) f32, reward ~ U(-1,1) (T, N) f32,
    terminated ~ Bernoulli(p) (T, N) bool.  ``device='cuda'`` draws on the GPU generator (bench
    inputs; not the CPU stream the parity tests use)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    g = torch.Generator(device=dev).manual_seed(seed)
    base_obs = torch.randn(horizon + 1, num_envs, obs_dim, generator=g, device=dev)
    base_reward = torch.rand(horizon, num_envs, generator=g, device=dev) * 2 - 1
    base_term = torch.rand(horizon, num_envs, generator=g, device=dev) < p_terminate
    return {"base_obs": base_obs, "base_reward": base_reward, "base_terminated": base_term}


class SyntheticVecEnvHelper:
    """EnvironmentHelper over the synthetic device VecEnv."""

    writes_into_buffer = True  # step(reward_out=, terminated_out=) / get_state(out=)
    graph_safe = True          # every step is device work on fixed buffers (hipGraph-capturable)

    def __init__(self, streams: Optional[dict] = None, run: Optional[Run] = None,
                 device: Optional[torch.device] = None, seed: int = 0, p_terminate: float = 0.0):
        self.rewards = []
        self.memory = []
        self.images = []
        self.run = run or Run.instance()
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self._streams = streams
        self._seed = seed
        self._p_terminate = p_terminate
        self.initialize()
        self.environment.timestep = self.timestep
        self.test_environment.timestep = self.test_timestep

    def initialize(self):
        ec, nc = self.run.environment_config, self.run.network_config
        n, t, o, w = ec.num_envs, ec.maximum_timesteps, nc.input_shape, ec.window_length
        self.num_envs, self.horizon, self.obs_dim, self.window = n, t, o, w
        streams = self._streams or make_synthetic_streams(n, t, o, self._seed, self._p_terminate)
        dev = self.device
        self.base_obs = streams["base_obs"].to(dev, torch.float32).contiguous()
        self.base_reward = streams["base_reward"].to(dev, torch.float32).contiguous()
        self.base_terminated = streams["base_terminated"].to(dev, torch.bool).contiguous()
        if self.base_obs.shape[0] < t + 1 or self.base_reward.shape[0] < t:
            raise ValueError("synthetic streams shorter than the horizon")
        f64 = dict(dtype=torch.float64, device=dev)
        self.timestep = Timestep(torch.zeros(n, o, w, **f64), torch.zeros(n, **f64),
                                 torch.zeros(n, dtype=torch.bool, device=dev),
                                 torch.zeros(n, dtype=torch.bool, device=dev), {})
        self.test_timestep = Timestep(torch.zeros(1, o, w, **f64), torch.zeros(1, **f64),
                                      torch.zeros(1, dtype=torch.bool, device=dev),
                                      torch.zeros(1, dtype=torch.bool, device=dev), {})
        self.environment = SimpleNamespace(num_envs=n)
        self.test_environment = SimpleNamespace(num_envs=1)
        self._obs_next = torch.empty(n, o, **f64)
        self._test_step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.t = 0

    # ---- EnvironmentHelper API -------------------------------------------------------------
    def reset(self, release_memory: bool = True):
        self.rewards = []
        if release_memory:
            self.memory = []
        self.images = []

    def reset_environment(self, test_phase: bool):
        """helper.py:59-67 + running_gym_sequential_vectorized.py:94-100.  The test env (env 0 of
        the streams) restarts at stream step 0 with every window slot = base_obs[0, 0]."""
        if test_phase:
            E.obs_window_push(self.test_timestep.observation, self.base_obs[0, :1].contiguous(),
                              all_reset=True)
            self.test_timestep.terminated.zero_()
            self.test_timestep.truncated.zero_()
            self._test_step.zero_()
            return
        self.t = 0
        E.obs_window_push(self.timestep.observation, self.base_obs[0], all_reset=True)
        self.timestep.terminated.zero_()
        self.timestep.truncated.zero_()

    def step(self, action: torch.Tensor, reward_out: Optional[torch.Tensor] = None,
             terminated_out: Optional[torch.Tensor] = None):
        """Training-phase step of all N envs (running_gym_sequential_vectorized.py:40-59, the window
        update of :53-58 / helper.py:51-57).
        ``reward_out`` / ``terminated_out`` let the engine land the outputs straight in its
        rollout buffer."""
        t = self.t
        if t >= self.horizon:
            raise RuntimeError("synthetic VecEnv: horizon exhausted; call reset_environment()")
        reward = reward_out if reward_out is not None else self.timestep.reward
        term = terminated_out if terminated_out is not None else self.timestep.terminated
        E.synthetic_env_step(self.base_obs[t + 1], self.base_reward[t], self.base_terminated[t],
                             action.contiguous(), self._obs_next, reward, term)
        E.obs_window_push(self.timestep.observation, self._obs_next, reset=term)
        self.timestep.reward = reward
        self.timestep.terminated = term
        self.t = t + 1

    def step_raw(self, action: torch.Tensor, reward_out: torch.Tensor,
                 terminated_out: torch.Tensor) -> torch.Tensor:
        """The physics half of :meth:`step`: advance the envs and return the new observation
        (N, O) f64 without pushing it into the window, so the engine's fused observe + act
        (ppo_observe_act) can push, standardise and act in one launch."""
        t = self.t
        if t >= self.horizon:
            raise RuntimeError("synthetic VecEnv: horizon exhausted; call reset_environment()")
        E.synthetic_env_step(self.base_obs[t + 1], self.base_reward[t], self.base_terminated[t],
                             action.contiguous(), self._obs_next, reward_out, terminated_out)
        self.timestep.reward = reward_out
        self.timestep.terminated = terminated_out
        self.t = t + 1
        return self._obs_next

    def get_state(self, test_phase: bool = False, out: Optional[torch.Tensor] = None):
        """(N, W, O) ``Run.dtype`` state (running_gym_sequential_vectorized.py:83-92)."""
        ts = self.test_timestep if test_phase else self.timestep
        n, o, w = ts.observation.shape
        if out is None:
            out = torch.empty(n, w, o, dtype=torch.float32, device=self.device)
        E.obs_normalize(ts.observation, out, normalize=self.run.normalize_observations)
        return out.view(n, w, o)

    def test_step(self, action: torch.Tensor, reward_sum: torch.Tensor) -> None:
        """One step of the evaluation env inside Algorithm.test (base_algorithm.py:30-39):
        test_environment.step(action.reshape(-1)), then reset_environment(test) on termination or
        shift + append otherwise, and rewards.append -- as one device launch
        (ppo_synthetic_test_step), the termination branch taken on the device.  ``reward_sum``
        (1,) f64 accumulates the rewards in order."""
        ts = self.test_timestep
        E.synthetic_test_step(self.base_obs, self.base_reward, self.base_terminated,
                              action.reshape(-1).contiguous(), ts.observation[0], self._test_step,
                              reward_sum, ts.terminated)

    def shift_observations(self, test_phase: bool, environment_index: int):
        ts = self.test_timestep if test_phase else self.timestep
        if test_phase:
            ts.observation[..., :-1] = ts.observation[..., 1:].clone()
        else:
            ts.observation[environment_index, :, :-1] = ts.observation[environment_index, :,
                                                                       1:].clone()


class HostPhysicsVecEnvHelper(SyntheticVecEnvHelper):
    """EnvironmentHelper whose physics runs on host cores (host_pool.HostPhysicsPool, P worker
    processes over env slices in shared memory), with the transfers the north_star names:
    actions device->host and observations / rewards / terminations host->device as
    hipMemcpyAsync on side streams between page-locked shared memory and the device.  Same
    dynamics and values as :class:`SyntheticVecEnvHelper` (tested bit-for-bit); not
    hipGraph-capturable (host work every step).

    overlap=True splits the envs into two halves with their own worker groups and side streams,
    and exposes the pipelined protocol PPOEngine's rollout drives (begin_half / release_half /
    finish_half): while one half steps its physics on the host, the GPU runs the other half's
    observe + act and both halves' DMAs, instead of serialising policy -> D2H -> physics -> H2D
    for all envs every step."""

    graph_safe = False

    def __init__(self, streams: Optional[dict] = None, run: Optional[Run] = None,
                 device: Optional[torch.device] = None, seed: int = 0, p_terminate: float = 0.0,
                 workers: int = 4, overlap: bool = True, step_delay: float = 0.0):
        self._workers = workers
        self._step_delay = step_delay  # test hook: seconds every worker sleeps per physics step
        self._overlap = overlap
        self.pool = None
        super().__init__(streams, run, device, seed, p_terminate)

    def initialize(self):
        from .host_pool import HostPhysicsPool
        super().initialize()  # device-side window / timestep buffers + device copies of streams
        lib = E._lib.load()
        if self.pool is not None:
            self.close()
        a = self.run.network_config.output_shape
        n = self.base_obs.shape[1]
        groups = 2 if (self._overlap and n >= 2 and self._workers >= 2) else 1
        self.pool = HostPhysicsPool(self.base_obs.cpu().numpy(), self.base_reward.cpu().numpy(),
                                    self.base_terminated.cpu().numpy(), a, self._workers,
                                    groups=groups, step_delay=self._step_delay)
        gb = self.pool.group_bounds
        self.halves = [(gb[g], gb[g + 1]) for g in range(self.pool.groups)]
        self._registered = []
        for key in ("action", "obs", "reward", "term"):
            arr = self.pool.v[key]
            E.check(lib.ppo_host_register(arr.ctypes.data, arr.nbytes))
            self._registered.append(arr.ctypes.data)
        self._sides = [torch.cuda.Stream(device=self.device) for _ in self.halves]
        self._side = self._sides[0]
        self._ev_d2h = [torch.cuda.Event() for _ in self.halves]
        self._lib = lib

    def close(self):
        if self.pool is None:
            return
        torch.cuda.synchronize(self.device)
        for p in getattr(self, "_registered", []):
            self._lib.ppo_host_unregister(p)
        self._registered = []
        self.pool.close()
        self.pool = None

    # ---- native pipelined rollout (ppo_host_rollout) --------------------------------------------
    def native_desc(self):
        """The pool as a ``ppo_host_pool_desc`` for the native rollout driver."""
        pool, v = self.pool, self.pool.v
        d = E._lib.HostPoolDesc()
        d.groups = pool.groups
        for g in range(pool.groups):
            d.group_lo[g], d.group_hi[g] = self.halves[g]
            ids = pool._group_workers[g]
            d.worker_lo[g], d.worker_hi[g] = ids[0], ids[-1] + 1
            d.gen[g] = pool._gen[g]
        d.ctrl, d.done = v["ctrl"].ctypes.data, v["done"].ctypes.data
        d.action, d.obs = v["action"].ctypes.data, v["obs"].ctypes.data
        d.reward, d.term = v["reward"].ctypes.data, v["term"].ctypes.data
        for key in ("action", "obs", "reward", "term"):
            dev = ctypes.c_void_p()
            E.check(self._lib.ppo_host_device_ptr(v[key].ctypes.data, ctypes.byref(dev)))
            setattr(d, key + "_dev", dev.value)
        return d

    def native_done(self, desc, reward_last: torch.Tensor, term_last: torch.Tensor) -> None:
        """Bookkeeping after a native rollout: the generations it advanced, the step counter."""
        for g in range(self.pool.groups):
            self.pool._gen[g] = int(desc.gen[g])
        self.t = self.horizon
        self.timestep.reward = reward_last
        self.timestep.terminated = term_last

    # ---- pipelined protocol (one half = one worker group + one side stream) -------------------
    def begin_half(self, g: int, action_rows: torch.Tensor) -> None:
        """Queue the D2H copy of half g's actions on its side stream, ordered after the work
        already enqueued on the current stream (call right after that half's observe + act)."""
        lo, hi = self.halves[g]
        v, side = self.pool.v, self._sides[g]
        side.wait_stream(torch.cuda.current_stream(self.device))
        act = action_rows.contiguous()
        nbytes = (hi - lo) * v["action"].shape[1] * 4
        E.check(self._lib.ppo_memcpy_async(v["action"][lo:hi].ctypes.data, act.data_ptr(), nbytes,
                                           2, side.cuda_stream))
        act.record_stream(side)
        self._ev_d2h[g].record(side)

    def release_half(self, g: int, t: int) -> None:
        """Host: wait for half g's actions to land, then start its workers on step t."""
        if self.t >= self.horizon:
            raise RuntimeError("host VecEnv: horizon exhausted; call reset_environment()")
        self._ev_d2h[g].synchronize()
        self.pool.release(g, t)

    def finish_half(self, g: int, reward_rows: torch.Tensor,
                    term_rows: torch.Tensor) -> torch.Tensor:
        """Wait for half g's workers, queue its H2D copies on its side stream and make the
        current stream wait for them; returns the half's (n_half, O) f64 observation rows."""
        lo, hi = self.halves[g]
        v, lib, side = self.pool.v, self._lib, self._sides[g]
        self.pool.wait(g)
        s = side.cuda_stream
        o = v["obs"].shape[1]
        obs_rows = self._obs_next[lo:hi]
        E.check(lib.ppo_memcpy_async(obs_rows.data_ptr(), v["obs"][lo:hi].ctypes.data,
                                     (hi - lo) * o * 8, 1, s))
        E.check(lib.ppo_memcpy_async(reward_rows.data_ptr(), v["reward"][lo:hi].ctypes.data,
                                     (hi - lo) * 8, 1, s))
        E.check(lib.ppo_memcpy_async(term_rows.data_ptr(), v["term"][lo:hi].ctypes.data,
                                     (hi - lo), 1, s))
        torch.cuda.current_stream(self.device).wait_stream(side)
        return obs_rows

    def end_step(self, reward_out: torch.Tensor, terminated_out: torch.Tensor) -> None:
        """Bookkeeping once every half has finished step t."""
        self.timestep.reward = reward_out
        self.timestep.terminated = terminated_out
        self.t += 1

    # ---- the unpipelined EnvironmentHelper.step protocol ---------------------------------------
    def _physics(self, action: torch.Tensor, reward_out: torch.Tensor,
                 terminated_out: torch.Tensor) -> None:
        if self.t >= self.horizon:
            raise RuntimeError("host VecEnv: horizon exhausted; call reset_environment()")
        t = self.t
        for g, (lo, hi) in enumerate(self.halves):
            self.begin_half(g, action[lo:hi])
        for g in range(len(self.halves)):
            self.release_half(g, t)
        for g, (lo, hi) in enumerate(self.halves):
            self.finish_half(g, reward_out[lo:hi], terminated_out[lo:hi])
        self.end_step(reward_out, terminated_out)

    def step(self, action: torch.Tensor, reward_out: Optional[torch.Tensor] = None,
             terminated_out: Optional[torch.Tensor] = None):
        reward = reward_out if reward_out is not None else self.timestep.reward
        term = terminated_out if terminated_out is not None else self.timestep.terminated
        self._physics(action, reward, term)
        E.obs_window_push(self.timestep.observation, self._obs_next, reset=term)

    def step_raw(self, action: torch.Tensor, reward_out: torch.Tensor,
                 terminated_out: torch.Tensor) -> torch.Tensor:
        self._physics(action, reward_out, terminated_out)
        return self._obs_next
