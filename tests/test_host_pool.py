"""Host physics pool on the CPU: P worker processes over shared memory
step the same values as a single-process evaluation of the synthetic dynamics, for any worker
count, including mid-trajectory terminations."""
import numpy as np
import pytest

from mujoco_reinforcement_learning_amd.host_pool import HostPhysicsPool, step_slice


def _streams(n=37, t=5, o=17, a=6, seed=0):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((t + 1, n, o)).astype(np.float32),
            (rng.random((t, n)) * 2 - 1).astype(np.float32),
            rng.random((t, n)) < 0.2, a)


def _reference(base_obs, base_reward, base_term, actions):
    """Plain numpy restatement of synthetic_env_step_kernel (scan_kernels.hip)."""
    n, o = base_obs.shape[1:]
    out = []
    for t, act in enumerate(actions):
        a64 = act.astype(np.float64)
        obs = np.empty((n, o))
        for f in range(o):
            obs[:, f] = base_obs[t + 1, :, f].astype(np.float64) + 0.1 * a64[:, f % act.shape[1]]
        ctrl = np.zeros(n)
        for j in range(act.shape[1]):
            ctrl = ctrl + a64[:, j] * a64[:, j]
        out.append((obs, base_reward[t].astype(np.float64) - 0.01 * ctrl, base_term[t].astype(np.uint8)))
    return out


@pytest.mark.parametrize("workers", [1, 3])
def test_pool_matches_single_process(workers):
    base_obs, base_reward, base_term, a = _streams()
    n = base_obs.shape[1]
    rng = np.random.default_rng(1)
    actions = [rng.standard_normal((n, a)).astype(np.float32) for _ in range(base_reward.shape[0])]
    ref = _reference(base_obs, base_reward, base_term, actions)
    pool = HostPhysicsPool(base_obs, base_reward, base_term, a, workers=workers)
    try:
        for t, act in enumerate(actions):
            pool.v["action"][...] = act
            pool.step(t)
            obs, rew, term = ref[t]
            assert np.array_equal(pool.v["obs"], obs)
            assert np.array_equal(pool.v["reward"], rew)
            assert np.array_equal(pool.v["term"], term)
    finally:
        pool.close()


def test_step_slice_partitions_compose():
    """Stepping [0, k) and [k, n) separately equals stepping [0, n) (what the workers rely on)."""
    base_obs, base_reward, base_term, a = _streams(n=20)
    n, o = base_obs.shape[1:]
    rng = np.random.default_rng(2)
    act = rng.standard_normal((n, a)).astype(np.float32)

    def views():
        return {"base_obs": base_obs, "base_reward": base_reward,
                "base_term": base_term.astype(np.uint8), "action": act.copy(),
                "obs": np.zeros((n, o)), "reward": np.zeros(n), "term": np.zeros(n, np.uint8)}
    whole, parts = views(), views()
    step_slice(whole, 2, 0, n)
    step_slice(parts, 2, 0, 7)
    step_slice(parts, 2, 7, n)
    for k in ("obs", "reward", "term"):
        assert np.array_equal(whole[k], parts[k])


def test_native_step_slice_matches_numpy():
    """The workers' C dynamics (libppo_hostenv.so) equal the numpy form bit for bit."""
    from mujoco_reinforcement_learning_amd._build import build_host_env
    from mujoco_reinforcement_learning_amd.host_pool import _native_step, step_slice_native
    build_host_env(verbose=False)
    fn = _native_step()
    assert fn is not None
    base_obs, base_reward, base_term, a = _streams(n=29, t=4)
    n, o = base_obs.shape[1:]
    rng = np.random.default_rng(3)

    def views():
        return {"base_obs": base_obs, "base_reward": base_reward,
                "base_term": base_term.astype(np.uint8),
                "action": rng.standard_normal((n, a)).astype(np.float32),
                "obs": np.zeros((n, o)), "reward": np.zeros(n), "term": np.zeros(n, np.uint8)}

    for t in range(base_reward.shape[0]):
        v1 = views()
        v2 = {k: x.copy() for k, x in v1.items()}
        step_slice(v1, t, 3, n - 2)
        step_slice_native(fn, v2, t, 3, n - 2)
        for k in ("obs", "reward", "term"):
            assert np.array_equal(v1[k], v2[k]), (t, k)
