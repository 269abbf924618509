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
    algo._finish_logging(algo.train(mem))  # the logged losses: all-reduced over the ranks
    if capture:
        return agent.packed_params().cpu(), mem["advantage"].cpu(), grads, agent, algo.last_losses
    return agent.packed_params().cpu(), mem["advantage"].cpu(), algo.last_losses


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    n_local = N_GLOBAL // world
    params, adv, losses = _run(n_local, (rank * n_local, (rank + 1) * n_local), "exact",
                               torch.device("cuda", 0))
    q.put((rank, params, adv, losses))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_exact_dp_two_ranks_match_single_process(gpu):
    p_single, adv_single, g_single, agent, loss_single = _run(N_GLOBAL, (0, N_GLOBAL), "local",
                                                              gpu, capture=True)
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
        r, params, adv, losses = q.get(timeout=300)
        got[r] = (params, adv, losses)
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
    # the logged losses (ppo.py:139-153): every rank reports the SUM over ranks of its shard's
    # terms, with the entropy bonus counted once (rank 0's share), i.e. the single process's loss
    print(f"exact DP x2 losses {got[0][2]} {got[1][2]} vs single {loss_single}")
    assert got[0][2] == got[1][2]
    for a, b in zip(got[0][2], loss_single):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), (got[0][2], loss_single)


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
    q.put((rank, agent.packed_params().cpu(), kernels, algo.last_losses))
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
    kernels = got[0][1]
    if shape == "wide":  # layered bf16-resident GEMMs, the fixed-order slab fold, Adam
        assert any(k.startswith("wide_gemm_kernel") for k in kernels), kernels
        assert "wide_reduce_kernel" in kernels and "wide_policy_fused_kernel" in kernels, kernels
        assert not any(k.startswith("fused_update_kernel") for k in kernels), kernels
        return
    # the data-parallel optimizer step: the fused kernel, reduce_slabs_kernel folding its slabs
    # into the flat gradient, the all-reduce,
    # then ONE tail launch: Adam + weight images + the next minibatch's gather
    assert any(k.startswith("fused_update_kernel") for k in kernels), kernels
    assert any(k.startswith("step_tail_kernel") for k in kernels), kernels
    assert "reduce_slabs_kernel" in kernels, kernels


def _ckpt_worker(rank, world, port, q, exp):
    """Local data parallel with the torch RNG (each rank its own forked generator): one
    iteration, agent.save(); then a fresh agent that load()s BEFORE its PPOEngine exists (the
    reference's order, main.py:117-124) must continue with the same per-rank generator."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.algorithm import PPOEngine
    from mujoco_reinforcement_learning_amd.environments import (SyntheticVecEnvHelper,
                                                                make_synthetic_streams)
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    dev = torch.device("cuda", 0)
    n, t, b = 16, 16, 64

    def build():
        s = make_synthetic_streams(n, t, 17, seed=41 + rank, p_terminate=0.05, device=dev)
        run = make_run(num_envs=n, horizon=t, hidden=(64, 64), batch_size=b, epochs=1, rng="torch",
                       seed=rank, dp_mode="local", experiment_path=exp)
        torch.manual_seed(0)
        agent = PPOEngineAgent(run, device=dev)
        return run, agent, s

    run, agent, s = build()
    algo = PPOEngine(SyntheticVecEnvHelper(s, run, device=dev), agent, log=lambda m: None)
    algo.iterate(verbose=False)
    ep = run.dynamic_config.current_episode
    run.dynamic_config.current_episode = ep - 1
    agent.save()
    torch.distributed.barrier()  # every rank's files written before anyone loads
    ahead = torch.randn(4, generator=algo._local_gen())  # the saved generator's next draws
    run2, agent2, s2 = build()
    run2.dynamic_config.current_episode = ep - 1
    agent2.load()  # no PPOEngine yet
    algo2 = PPOEngine(SyntheticVecEnvHelper(s2, run2, device=dev), agent2, log=lambda m: None)
    got = torch.randn(4, generator=algo2._local_gen())
    files = sorted(f for f in os.listdir(f"{exp}/networks/{ep - 1}") if f.startswith("engine_rng"))
    q.put((rank, torch.equal(ahead, got), files))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_local_dp_checkpoint_round_trip_per_rank_generators(gpu, tmp_path):
    """each rank's generator goes to its own file (engine_rng_rank{r}.pth) and a
    resumed rank continues its own stream, also when load() runs before PPOEngine exists."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    exp = str(tmp_path / "exp")
    procs = [ctx.Process(target=_ckpt_worker, args=(r, 2, port, q, exp)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        r, same, files = q.get(timeout=300)
        got[r] = (same, files)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert got[r][0], f"rank {r} did not resume its own generator"
        assert got[r][1] == ["engine_rng_rank0.pth", "engine_rng_rank1.pth"], got[r][1]


def _rccl_worker(q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
                      WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.distributed.init_process_group("nccl", device_id=dev)
    from mujoco_reinforcement_learning_amd.distributed import DataParallel
    x = torch.arange(142605, dtype=torch.float32, device=dev) * 0.5  # the 2x256 flat gradient size
    want = x.clone()
    torch.distributed.all_reduce(x, op=torch.distributed.ReduceOp.SUM)
    DataParallel().allreduce_grad(x)  # world 1: no collective
    torch.cuda.synchronize()
    q.put((torch.equal(x.cpu(), want.cpu()), torch.distributed.get_backend()))
    torch.distributed.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_rccl_allreduce_known_answer(gpu):
    """RCCL ("nccl" backend on ROCm) initialises on the device and an all-reduce of a
    flat-gradient-sized buffer returns the known sum (one GPU on this box: world 1)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(q,))
    p.start()
    ok, backend = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0 and ok and backend == "nccl"


def test_bench_self_launches_two_ranks_on_one_gpu(gpu):
    """``python bench.py --gpus 2`` as a plain invocation (the driver's scaling run)
    starts its own two ranks; here both share cuda:0 over gloo (PPO_BENCH_ONE_DEVICE=1) on a tiny
    workload, and rank 0 prints one JSON line with n_gpus 2."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PPO_BENCH_BACKEND="gloo", PPO_BENCH_ONE_DEVICE="1")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps",
                        "2", "--warmup", "1", "--num-envs", "64", "--horizon", "16", "--batch",
                        "256", "--epochs", "1", "--no-cpu-baseline", "--no-legs"], env=env,
                       capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    print(f"bench --gpus 2 (one GPU, gloo): {rec['value']:.4g} env-steps/s, "
          f"{rec['ms_per_step']:.2f} ms/step")
    assert rec["n_gpus"] == 2 and rec["value"] > 0 and rec["steps"] == 2


def _graph_dp_worker(q):
    """World-1 nccl process group: the data-parallel step sequence (fused gradient -> native RCCL
    all-reduce -> Adam tail) captured in one hipGraph (PPO_DP_REHEARSE=rccl) against the same
    sequence run eagerly with a no-op exchange (PPO_DP_REHEARSE=1), then the all-reduce's per-call
    cost on this GPU at the 2x256 and Humanoid 3x512 flat-gradient sizes."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
                      WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.distributed.init_process_group("nccl", device_id=dev)
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.algorithm import PPOEngine
    from mujoco_reinforcement_learning_amd.environments import (SyntheticVecEnvHelper,
                                                                make_synthetic_streams)
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    out = {}
    for mode in ("1", "rccl"):
        os.environ["PPO_DP_REHEARSE"] = mode
        s = make_synthetic_streams(64, 16, 17, seed=41, p_terminate=0.05, device=dev)
        run = make_run(num_envs=64, horizon=16, hidden=(256, 256), batch_size=256, epochs=2,
                       rng="philox", seed=3, dp_mode="local", precision="bf16")
        torch.manual_seed(0)
        agent = PPOEngineAgent(run, device=dev)
        algo = PPOEngine(SyntheticVecEnvHelper(s, run, device=dev), agent, log=lambda m: None)
        for _ in range(3):  # eager warm-up, capture + replay, replay
            algo.iterate(verbose=False)
        torch.cuda.synchronize()
        out[mode] = (agent.packed_params().cpu(), algo.dp.comm is not None,
                     getattr(algo, "_tg_graph", None) is not None, algo.last_losses)
        if algo.dp.comm is not None:
            algo.dp.comm.check()
            comm = algo.dp.comm
    del os.environ["PPO_DP_REHEARSE"]
    # per-call cost of the native all-reduce (world 1: RCCL's launch / proxy floor)
    times = {}
    for n in (142605, 1445923):  # 2x256 HalfCheetah, 3x512 Humanoid flat gradients
        x = torch.ones(n, dtype=torch.float32, device=dev)
        for _ in range(20):
            comm.allreduce(x)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            comm.allreduce(x)
        e1.record()
        torch.cuda.synchronize()
        eager_us = e0.elapsed_time(e1) * 1e3 / 200
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for _ in range(100):
                comm.allreduce(x)
        g.replay()
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        times[n] = (eager_us, e0.elapsed_time(e1) * 1e3 / 100, bool(torch.all(x == 1.0)))
    q.put((out, times))
    torch.distributed.destroy_process_group()


def test_dp_step_graph_captured_with_rccl_allreduce(gpu):
    """VERDICT r04 item 4 / SURVEY s8(e): the data-parallel optimizer loop with the native RCCL
    all-reduce (csrc/comm.hip, ppo_allreduce_grads on the ctx's communicator) captured inside the
    hipGraph is bitwise equal to the eager DP sequence; per-call all-reduce times printed."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_graph_dp_worker, args=(q,))
    p.start()
    out, times = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    p_eager, comm_eager, graph_eager, loss_eager = out["1"]
    p_graph, comm_graph, graph_graph, loss_graph = out["rccl"]
    assert not comm_eager and not graph_eager
    assert comm_graph and graph_graph, "the rccl rehearsal did not capture the DP loop"
    assert torch.equal(p_eager, p_graph)
    assert loss_eager == loss_graph
    for n, (eager_us, graph_us, ok) in times.items():
        print(f"native RCCL all-reduce, world 1, {n * 4 / 1e6:.2f} MB: eager {eager_us:.2f} us, "
              f"in a hipGraph {graph_us:.2f} us per call")
        assert ok
