"""GPU: the engine's exact data-parallel mode, 2 ranks (gloo, both on cuda:0 -- the box has one
GPU; RCCL is the same code path with backend "nccl") against a single-process run over all envs.

Each rank owns half of the 16 envs, replays the global reference RNG stream (eps rows of its shard,
the global randperm filtered to its shard, ppo.py:103-110) and all-reduces the flat gradient once
per optimizer step.  Post-iteration parameters must match the single process up to the summation
order of the gradient (2 partial sums vs 1).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from parity_util import assert_params_match, capture_engine_grads

pytestmark = pytest.mark.gpu

N_GLOBAL, T, B, EPOCHS = 16, 16, 64, 2


def _streams():
    from mujoco_reinforcement_learning_amd.environments import make_synthetic_streams
    return make_synthetic_streams(N_GLOBAL, T, 17, seed=21, p_terminate=0.05)


def _run(n_envs, shard, dp_mode, dev, capture=False):
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.algorithm import PPOEngine
    from mujoco_reinforcement_learning_amd.environments import SyntheticVecEnvHelper
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    s = _streams()
    lo, hi = shard
    s = {k: v[:, lo:hi].contiguous() for k, v in s.items()}
    run = make_run(num_envs=n_envs, horizon=T, hidden=(64, 64), batch_size=B, epochs=EPOCHS,
                   rng="torch", dp_mode=dp_mode)
    torch.manual_seed(0)
    agent = PPOEngineAgent(run, device=dev, max_rows=max(B, n_envs))
    algo = PPOEngine(SyntheticVecEnvHelper(s, run, device=dev), agent, log=lambda m: None)
    torch.manual_seed(1234)
    mem = algo.rollout()
    algo.calculate_advantages(mem)
    grads = capture_engine_grads(algo) if capture else None
    algo.train(mem)
    if capture:
        return agent.packed_params().cpu(), mem["advantage"].cpu(), grads, agent
    return agent.packed_params().cpu(), mem["advantage"].cpu()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    n_local = N_GLOBAL // world
    params, adv = _run(n_local, (rank * n_local, (rank + 1) * n_local), "exact",
                       torch.device("cuda", 0))
    q.put((rank, params, adv))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_exact_dp_two_ranks_match_single_process(gpu):
    p_single, adv_single, g_single, agent = _run(N_GLOBAL, (0, N_GLOBAL), "local", gpu,
                                                 capture=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        r, params, adv = q.get(timeout=300)
        got[r] = (params, adv)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # replicas identical to each other (same all-reduced grads, same Adam)
    assert torch.equal(got[0][0], got[1][0])
    # rollout/GAE per shard: rank r's advantages are the single run's env rows [r*8, (r+1)*8)
    torch.testing.assert_close(torch.cat([got[0][1], got[1][1]]), adv_single, rtol=1e-5,
                               atol=1e-5)
    # the single process is the reference here: rtol 1e-5 except the counted Adam sign-flip-prone
    # set (gradient below 1e-3 of its tensor's max at some step; tests/parity_util.py)
    assert_params_match(got[0][0], p_single, g_single, agent, 1e-4, label="exact DP x2")


_LOCAL_SHAPES = {  # name -> (hidden, obs, act)
    "fused": ((256, 256), 17, 6),           # fused_update_kernel (HalfCheetah shapes)
    "wide": ((512, 512, 512), 376, 17)}     # the wide bf16 path (Humanoid, BASELINE configs[3])


def _local_worker(rank, world, port, q, shape="fused"):
    """Weak-scaling ("local") data parallel on the bf16 paths: each rank its own env shard and
    Philox shuffles; per step the gradient, the all-reduce, Adam (+ images + next gather on the
    fused path).  Returns the parameters after two iterations and the kernels that ran."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.algorithm import PPOEngine
    from mujoco_reinforcement_learning_amd.environments import (SyntheticVecEnvHelper,
                                                                make_synthetic_streams)
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    dev = torch.device("cuda", 0)
    n, t, b = 64, 16, 256
    hidden, obs, act = _LOCAL_SHAPES[shape]
    s = make_synthetic_streams(n, t, obs, seed=31 + rank, p_terminate=0.05, device=dev)
    run = make_run(num_envs=n, horizon=t, hidden=hidden, batch_size=b, epochs=2, obs_dim=obs,
                   act_dim=act, rng="philox", seed=rank, dp_mode="local", precision="bf16")
    torch.manual_seed(0)
    agent = PPOEngineAgent(run, device=dev)
    algo = PPOEngine(SyntheticVecEnvHelper(s, run, device=dev), agent, log=lambda m: None)
    agent.engine.timing(True, capacity=4096)
    for _ in range(2):
        algo.iterate(verbose=False)
    torch.cuda.synchronize()
    kernels = sorted(agent.engine.timing_kernels())
    agent.engine.timing(False)
    q.put((rank, agent.packed_params().cpu(), (kernels, agent.engine.fused_fold()),
           algo.last_losses))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("shape", ["fused", "wide"])
def test_local_dp_two_ranks_fused_replicas_agree(gpu, shape):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_local_worker, args=(r, 2, port, q, shape)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        r, params, kernels, losses = q.get(timeout=300)
        got[r] = (params, kernels, losses)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # replicas bit-identical (same all-reduced gradient, same Adam), and they moved
    assert torch.equal(got[0][0], got[1][0])
    assert all(abs(x) < 1e6 for x in got[0][2])
    kernels, fold = got[0][1]
    if shape == "wide":  # layered bf16-resident GEMMs, the fixed-order slab fold, Adam
        assert any(k.startswith("wide_gemm_kernel") for k in kernels), kernels
        assert "wide_reduce_kernel" in kernels and "wide_policy_fused_kernel" in kernels, kernels
        assert not any(k.startswith("fused_update_kernel") for k in kernels), kernels
        return
    # the data-parallel optimizer step: the fused kernel (slabs folded to the flat gradient in
    # the same launch, or by reduce_slabs_kernel without the in-launch fold), the all-reduce,
    # then ONE tail launch: Adam + weight images + the next minibatch's gather
    assert any(k.startswith("fused_update_kernel") for k in kernels), kernels
    assert "step_tail_kernel" in kernels, kernels
    assert ("reduce_slabs_kernel" in kernels) == (not fold), (fold, kernels)
