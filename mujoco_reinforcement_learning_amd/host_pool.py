"""Host physics pool (BASELINE north_star: "MuJoCo physics itself stays on
the host cores as a vectorized subprocess pool with pinned hipMemcpyAsync obs->GPU / action->CPU
overlapped on a side stream").

The reference steps its VecEnv in-process (``running_gym_sequential_vectorized.py:21-59``:
``gymnasium.make_vec`` + a per-env Python window loop).  Here P worker processes each own a
contiguous slice of the N envs.  All per-step arrays live in POSIX shared memory that the GPU side
page-locks (``ppo_host_register``):
- actions (N, A) f32, written by a device->host DMA;
- next observations (N, O) f64, rewards (N,) f64 and terminations (N,) u8, read back by
  host->device DMAs.

The workers form ``groups`` independent groups over contiguous env ranges (one control word each),
so the caller can pipeline: while group 0 steps its envs on the host, the GPU runs group 1's
policy and DMAs, and the other way round (environments.HostPhysicsVecEnvHelper, overlap mode).
One group step is: DMA the group's actions down, release its workers (a generation word in shared
memory), every worker advances its slice and publishes its done word, DMA the results up.
Hand-offs spin on those words (yielding the core), so a step costs microseconds of
synchronisation rather than a semaphore round trip.  Workers import numpy only and never touch
the GPU.

Physics: gymnasium / mujoco are not installed in this image, so the workers run the engine's
synthetic dynamics (``environments.py`` docstring; bit-identical to
``synthetic_env_step_kernel``):

    obs'      = base_obs[t+1] + 0.1 * a[:, o % A]      (f64)
    reward    = base_reward[t] - 0.01 * sum_a a^2      (f64, summed in order)
    terminated = base_terminated[t]

``step_slice`` is the one function a real MuJoCo pool replaces: it would call ``env.step`` on the
worker's gymnasium envs.
"""
from __future__ import annotations

import ctypes
import multiprocessing as mp
import os
import time
from multiprocessing import shared_memory
from typing import Dict, Tuple

import numpy as np

# ctrl words per group: step index, stop flag, step generation (bumped by the host to release it)
_CTRL_T, _CTRL_STOP, _CTRL_GEN = 0, 1, 2


def _attach(specs: Dict[str, Tuple[str, tuple, str]]):
    shms, views = [], {}
    for key, (name, shape, dtype) in specs.items():
        shm = shared_memory.SharedMemory(name=name)
        shms.append(shm)
        views[key] = np.ndarray(shape, dtype=np.dtype(dtype), buffer=shm.buf)
    return shms, views


_HOSTENV = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libppo_hostenv.so")


def _native_step():
    """The C form of step_slice (csrc/host/synthetic_physics.c -> libppo_hostenv.so), or None
    when the library is not built (numpy form below; same values)."""
    if not os.path.exists(_HOSTENV):
        return None
    fn = ctypes.CDLL(_HOSTENV).ppo_host_step_slice
    fn.restype = None
    fn.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int64, ctypes.c_int64]
    return fn


def step_slice_native(fn, v: Dict[str, np.ndarray], t: int, lo: int, hi: int) -> None:
    n, o = v["obs"].shape
    fn(v["base_obs"].ctypes.data, v["base_reward"].ctypes.data, v["base_term"].ctypes.data,
       v["action"].ctypes.data, v["obs"].ctypes.data, v["reward"].ctypes.data,
       v["term"].ctypes.data, n, o, v["action"].shape[1], t, lo, hi)


def step_slice(v: Dict[str, np.ndarray], t: int, lo: int, hi: int) -> None:
    """Advance envs [lo, hi) by one step (the synthetic dynamics above)."""
    a = v["action"][lo:hi].astype(np.float64)
    n_act = a.shape[1]
    o = v["obs"].shape[1]
    v["obs"][lo:hi] = v["base_obs"][t + 1, lo:hi].astype(np.float64) + 0.1 * a[:, np.arange(o) % n_act]
    ctrl = np.zeros(hi - lo)
    for j in range(n_act):  # in order, as the kernel's loop
        ctrl = ctrl + a[:, j] * a[:, j]
    v["reward"][lo:hi] = v["base_reward"][t, lo:hi].astype(np.float64) - 0.01 * ctrl
    v["term"][lo:hi] = v["base_term"][t, lo:hi]


def _wait_change(word: np.ndarray, idx: int, old: int, stop: np.ndarray = None) -> int:
    """Spin (yielding the core) until word[idx] != old; a step hand-off costs microseconds
    instead of a semaphore round trip."""
    while True:
        cur = int(word[idx])
        if cur != old or (stop is not None and stop[_CTRL_STOP]):
            return cur
        time.sleep(0)


def _worker(wid: int, grp: int, lo: int, hi: int, specs, step_delay: float = 0.0) -> None:
    shms, v = _attach(specs)
    ctrl, done = v["ctrl"][grp], v["done"]
    native = _native_step()
    gen = 0
    try:
        while True:
            gen = _wait_change(ctrl, _CTRL_GEN, gen, stop=ctrl)
            if ctrl[_CTRL_STOP]:
                break
            if native is not None:
                step_slice_native(native, v, int(ctrl[_CTRL_T]), lo, hi)
            else:
                step_slice(v, int(ctrl[_CTRL_T]), lo, hi)
            if step_delay > 0:  # test hook: a slow physics step (the native driver's watchdog)
                time.sleep(step_delay)
            done[wid] = gen  # publish after the slice's outputs are written
    finally:
        for s in shms:
            s.close()


class HostPhysicsPool:
    """P worker processes stepping env slices in shared memory (see the module docstring)."""

    def __init__(self, base_obs: np.ndarray, base_reward: np.ndarray, base_term: np.ndarray,
                 act_dim: int, workers: int = 4, groups: int = 1, step_delay: float = 0.0):
        t1, n, o = base_obs.shape
        self.num_envs, self.obs_dim, self.act_dim = n, o, act_dim
        self.groups = max(1, min(int(groups), n))
        self.workers = max(self.groups, min(int(workers), n))
        self.workers -= self.workers % self.groups  # equal worker count per group
        arrays = {
            "base_obs": (base_obs.shape, "float32"),
            "base_reward": (base_reward.shape, "float32"),
            "base_term": (base_term.shape, "uint8"),
            "action": ((n, act_dim), "float32"),
            "obs": ((n, o), "float64"),
            "reward": ((n,), "float64"),
            "term": ((n,), "uint8"),
            "ctrl": ((self.groups, 3), "int64"),
            "done": ((self.workers,), "int64"),
        }
        self._shms, self.specs, self.v = [], {}, {}
        for key, (shape, dtype) in arrays.items():
            nbytes = max(1, int(np.prod(shape)) * np.dtype(dtype).itemsize)
            shm = shared_memory.SharedMemory(create=True, size=nbytes)
            self._shms.append(shm)
            self.specs[key] = (shm.name, shape, dtype)
            self.v[key] = np.ndarray(shape, dtype=np.dtype(dtype), buffer=shm.buf)
        self.v["base_obs"][...] = base_obs
        self.v["base_reward"][...] = base_reward
        self.v["base_term"][...] = base_term.astype(np.uint8)
        self.v["ctrl"][...] = 0
        self.v["done"][...] = 0
        self._gen = [0] * self.groups
        ctx = mp.get_context("spawn")  # never fork a process that may have initialised HIP
        self.group_bounds = [int(x) for x in np.linspace(0, n, self.groups + 1).astype(int)]
        per = self.workers // self.groups
        self._procs, self._group_workers = [], []
        for g in range(self.groups):
            lo, hi = self.group_bounds[g], self.group_bounds[g + 1]
            wb = np.linspace(lo, hi, per + 1).astype(int)
            ids = list(range(g * per, (g + 1) * per))
            self._group_workers.append(ids)
            for k, wid in enumerate(ids):
                self._procs.append(ctx.Process(target=_worker, daemon=True,
                                               args=(wid, g, int(wb[k]), int(wb[k + 1]),
                                                     self.specs, float(step_delay))))
        for p in self._procs:
            p.start()
        self._closed = False

    def release(self, group: int, t: int) -> None:
        """Start step t of the group's envs (its workers read v['action'] rows of the group)."""
        self._gen[group] += 1
        ctrl = self.v["ctrl"][group]
        ctrl[_CTRL_T] = t
        ctrl[_CTRL_GEN] = self._gen[group]  # release (after the step index and the actions)

    def wait(self, group: int) -> None:
        """Block until the group's workers have published step results (obs / reward / term)."""
        done, ids = self.v["done"], self._group_workers[group]
        lo, hi = ids[0], ids[-1] + 1
        gen = self._gen[group]
        deadline, spins = time.monotonic() + 60.0, 0
        while int(done[lo:hi].min()) != gen:
            spins += 1
            if spins % 4096 == 0 and (time.monotonic() > deadline or
                                      not all(p.is_alive() for p in self._procs)):
                raise RuntimeError("host physics pool: a worker died or stalled")
            time.sleep(0)

    def step(self, t: int) -> None:
        """Advance all envs from step t (every group, then wait for all)."""
        for g in range(self.groups):
            self.release(g, t)
        for g in range(self.groups):
            self.wait(g)

    def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        self.v["ctrl"][:, _CTRL_STOP] = 1
        for p in self._procs:
            p.join(timeout=10)
            if p.is_alive():
                p.terminate()
        self.v = {}
        for s in self._shms:
            s.close()
            s.unlink()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
