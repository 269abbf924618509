#!/usr/bin/env python
"""bench.py -- env-steps/sec of the PPO iteration on N MI355X GPUs (BASELINE.json metric).

One "step" = one full PPO iteration of the hot path on each rank: T=128 sequential rollout steps
over N=4096 synthetic envs (device dynamics + obs standardisation + actor/critic forward +
sampling + log-prob), GAE + value targets, then E=10 epochs x 8 minibatches of 65,536 rows
(actor/critic forward + loss + backward + fused Adam; for N_gpus > 1 one RCCL all-reduce of the
flat gradient per optimizer step).  Inputs are resident in HBM before timing starts.
value = N_gpus * 4096 * 128 * steps / max-over-ranks wall time (weak scaling: envs per GPU fixed).

Also reported on the same JSON line:
  roofline      the dominant kernel instantiation (most device time in the timed region), from
                HIP events on its dispatch packets (hipExtLaunchKernelGGL) recorded live:
                algorithmic FLOPs or bytes per launch / mean launch time vs the MI355X peak;
                `kernel` is its rocprofv3 name; `traffic` = PMC HBM bytes per launch from
                profiles/traffic.json when present (same command under rocprofv3 --pmc)
  gae_roofline  the same for the GAE scan (north-star >= 40 % HBM target)
  cpu_baseline  the oracle (oracle/ppo_ref.py, torch-CPU restatement of ppo.py) on a bounded
                sample of the same workload, on rank 0 at N_gpus = 1 only
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

METRIC = "env-steps/sec (whole node) HalfCheetah-v4 4096 envs at 1/2/4/8 MI355X"
# separate measurements (not the headline): their own metric strings
METRICS = {"mlp": METRIC,
           "lstm": "env-steps/sec main.py BiLSTM actor-critic (O=348, W=5, latent 256), 1024 envs, "
                   "1x MI355X",
           "cnn": "env-steps/sec dm_control cheetah-run pixels 84x84x3, 1024 envs, small CNN encoder "
                  "(Nature-DQN), 1x MI355X"}
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: F32 MFMA = vector peak (dense)
PEAK_BF16_MFMA_TFLOPS = 2516.6  # MI355X_MICROARCH.md: bf16 dense (2.5 PF; sparsity excluded)
PEAK_HBM_GBS = 8000.0           # MI355X HBM3E spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--model", choices=("mlp", "lstm", "cnn"), default="mlp",
                   help="mlp: the north_star MLP actor-critic (the headline metric); lstm: the "
                        "reference PPOAgent's BiLSTM actor / critic on main.py's network (O=348, "
                        "W=5, latent 256, [256,256,128,128], A=17) at N=1024, B=16384; cnn: "
                        "BASELINE configs[4], 84x84x3 pixel frames, Nature-DQN encoder + 2x256 "
                        "heads, A=6, N=1024, B=16384 (unless overridden) -- separate "
                        "measurements, not the headline line")
    p.add_argument("--window", type=int, default=None)
    p.add_argument("--latent", type=int, default=256)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--num-envs", type=int, default=4096)
    p.add_argument("--horizon", type=int, default=128)
    p.add_argument("--obs-dim", type=int, default=17)
    p.add_argument("--act-dim", type=int, default=6)
    p.add_argument("--hidden", type=str, default="256,256")
    p.add_argument("--batch", type=int, default=65536)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--rng", choices=("philox", "torch"), default="philox")
    p.add_argument("--precision", choices=("f32", "bf16"), default="bf16",
                   help="fc-layer GEMM precision: bf16 (default; bf16 operands, f32 accumulate, f32 "
                        "master params -- BASELINE.json configs[1]) or f32 (bit-level parity "
                        "mode with the reference's f32 CPU trainer)")
    p.add_argument("--cpu-baseline", dest="cpu_baseline", action="store_true", default=True)
    p.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    p.add_argument("--cpu-rollout-steps", type=int, default=128)
    p.add_argument("--cpu-epochs", type=int, default=1)
    p.add_argument("--no-timing", action="store_true", help="skip per-kernel event timing")
    p.add_argument("--timing-iters", type=int, default=2,
                   help="eager iterations after the timed region that carry per-kernel events")
    p.add_argument("--env", choices=("device", "host"), default="device",
                   help="device: synthetic dynamics on the GPU (the measured default); host: the "
                        "same dynamics in a host worker pool with pinned async copies (PCIe-inclusive)")
    p.add_argument("--env-workers", type=int, default=8, help="host pool worker processes")
    p.add_argument("--no-legs", action="store_true",
                   help="skip the extra same-workload legs (f32 precision, host-pool env) that the "
                        "default N=1 line carries next to `value`")
    p.add_argument("--leg-steps", type=int, default=3, help="timed iterations per extra leg")
    p.add_argument("--no-graphs", action="store_true",
                   help="launch the rollout and the update loop eagerly (no hipGraph replay)")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py output)")
    args = p.parse_args()
    if args.model == "lstm":
        defaults = {"num_envs": 1024, "obs_dim": 348, "act_dim": 17, "hidden": "256,256,128,128",
                    "batch": 16384, "window": 5}
        for k, v in defaults.items():
            if getattr(args, k) == p.get_default(k):
                setattr(args, k, v)
        args.no_timing = True  # per-kernel times for this leg come from rocprofv3
        args.no_legs = True
        args.cpu_baseline = False
    if args.model == "cnn":
        defaults = {"num_envs": 1024, "obs_dim": 84 * 84 * 3, "act_dim": 6, "batch": 16384}
        for k, v in defaults.items():
            if getattr(args, k) == p.get_default(k):
                setattr(args, k, v)
        args.no_legs = True
    if args.window is None:
        args.window = 1
    return args


def load_traffic(path):
    """{kernel name: HBM bytes per launch} from a PMC pass over this same command
    (tools/pmc_traffic.py; FETCH_SIZE x2 + WRITE_SIZE per MI355X_MICROARCH.md), or {}."""
    if not path or not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f).get("bytes_per_launch", {})


# gymnasium observation / action sizes of the BASELINE configs (SURVEY.md s8 notation)
_ENV_NAMES = {(17, 6): "HalfCheetah-v4", (27, 8): "Ant-v4", (376, 17): "Humanoid-v4",
              (348, 17): "main.py humanoid (O=348)", (84 * 84 * 3, 6): "cheetah-run pixels"}


def roofline(name, c, traffic, force_hbm=False):
    """Roofline of one kernel instantiation from its live event records.  The bound is the roof
    the kernel's own algorithmic work hits first: MFMA (FLOPs / dense peak of its dtype) or HBM
    (bytes / 8 TB/s); achieved = that work per launch / mean launch duration."""
    launches = max(c["launches"], 1)
    avg_s = c["ms"] * 1e-3 / launches
    # the fused update kernel and the wide path's GEMMs are bf16-only; the layered GEMMs carry
    # their dtype in the name
    bf16 = "bf16" in name or "wide_gemm" in name or c["class"] == "fused_update"
    peak_f = PEAK_BF16_MFMA_TFLOPS if bf16 else PEAK_FP32_MFMA_TFLOPS
    t_mfma = c["flops"] / (peak_f * 1e12)
    t_hbm = c["bytes"] / (PEAK_HBM_GBS * 1e9)
    mfma = (c["class"].startswith("gemm") or c["class"] in ("fused_update", "conv")) and \
        t_mfma >= t_hbm and not force_hbm
    if mfma:
        achieved, peak, unit = c["flops"] / launches / avg_s / 1e12, peak_f, "TFLOP/s"
    else:
        achieved, peak, unit = c["bytes"] / launches / avg_s / 1e9, PEAK_HBM_GBS, "GB/s"
    return {"bound": "mfma" if mfma else "hbm", "kernel": name, "achieved": achieved,
            "peak": peak, "unit": unit, "frac": achieved / peak,
            "traffic": traffic.get(name), "avg_launch_us": avg_s * 1e6, "launches": c["launches"],
            "algorithmic_per_launch": (c["flops"] if mfma else c["bytes"]) / launches}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> int:
    """The cores this process may really use: its affinity set, capped by the cgroup CPU quota
    (a GPU box's affinity lists the whole machine while its quota is a share of it) and by
    OMP_NUM_THREADS when the environment sets one."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def _progress(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(args, hidden):
    """Oracle on the host cores: rollout_steps of the T-step rollout, the full GAE, cpu_epochs of
    the E-epoch update; extrapolated linearly to one full iteration."""
    from oracle import ppo_ref as R
    threads = cpu_share()  # every core this process may use
    torch.set_num_threads(threads)
    _progress(f"cpu baseline on {threads} threads ({cpu_model()})")
    n, t = args.num_envs, args.horizon
    cfg = R.RefConfig(num_envs=n, horizon=t, obs_dim=args.obs_dim, act_dim=args.act_dim,
                      actor_hidden=hidden, critic_hidden=hidden, batch_size=args.batch,
                      epochs=args.cpu_epochs)
    g = torch.Generator().manual_seed(0)
    env = R.RefSyntheticEnv(torch.randn(t + 1, n, args.obs_dim, generator=g),
                            torch.rand(t, n, generator=g) * 2 - 1,
                            torch.zeros(t, n, dtype=torch.bool), 1, args.act_dim)
    torch.manual_seed(0)
    agent = R.RefAgent(cfg)
    k = min(args.cpu_rollout_steps, t)
    cfg.horizon = k
    t0 = time.perf_counter()
    mem = R.rollout(env, agent)  # k steps
    t_roll = (time.perf_counter() - t0) * (t / k)
    _progress(f"cpu baseline rollout: {k} steps in {t_roll * k / t:.2f} s")
    cfg.horizon = t
    # full-size buffer for GAE / update: tile the k sampled steps to T
    reps = (t + k - 1) // k
    full = {key: v.repeat(1, reps, *([1] * (v.dim() - 2)))[:, :t].contiguous()
            for key, v in mem.items()}
    t0 = time.perf_counter()
    R.calculate_advantages(full, cfg)
    t_gae = time.perf_counter() - t0
    t0 = time.perf_counter()
    R.train(agent, full, 0)
    t_epoch = (time.perf_counter() - t0) / args.cpu_epochs
    _progress(f"cpu baseline update: {args.cpu_epochs} epoch(s) in {t_epoch * args.cpu_epochs:.2f} s")
    t_iter = t_roll + t_gae + t_epoch * args.epochs
    return {"value": n * t / t_iter, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "torch": torch.__version__,
            "sample": (f"oracle/ppo_ref.py, the torch-CPU restatement of ppo.py (the reference itself "
                       f"was not run: its PPO modules import tensordict / torchrl, which are not "
                       f"installed; torch {torch.__version__} CPU, {threads} threads): "
                       f"{k} of {t} rollout steps + full GAE + {args.cpu_epochs} of {args.epochs} "
                       f"epochs at N={n}, B={args.batch}, 2x{hidden[0]} MLP; extrapolated "
                       f"(rollout {t_roll:.2f}s, gae {t_gae:.3f}s, epoch {t_epoch:.2f}s/iter-scaled)"),
            "seconds_per_iteration": t_iter}


def cpu_baseline_cnn(args, hidden):
    """The pixel oracle (oracle/cnn_ref.py) on the host cores: rollout_steps of the T-step
    rollout, the full GAE and ONE minibatch of the E x M update, extrapolated to one iteration."""
    from oracle import cnn_ref as C
    from oracle import ppo_ref as R
    threads = cpu_share()
    torch.set_num_threads(threads)
    _progress(f"cpu baseline (cnn) on {threads} threads ({cpu_model()})")
    n, t, b = args.num_envs, args.horizon, args.batch
    cfg = R.RefConfig(num_envs=n, horizon=t, act_dim=args.act_dim, actor_hidden=hidden,
                      critic_hidden=hidden, batch_size=b, epochs=1)
    g = torch.Generator().manual_seed(0)
    env = C.RefPixelEnv(0, torch.rand(t, n, generator=g) * 2 - 1,
                        torch.zeros(t, n, dtype=torch.bool), args.act_dim)
    torch.manual_seed(0)
    agent = C.RefCNNAgent(cfg)
    k = min(args.cpu_rollout_steps, 4, t)
    cfg.horizon = k
    t0 = time.perf_counter()
    mem = R.rollout(env, agent)
    t_roll = (time.perf_counter() - t0) * (t / k)
    cfg.horizon = t
    reps = (t + k - 1) // k
    full = {key: v.repeat(1, reps, *([1] * (v.dim() - 2)))[:, :t].contiguous()
            for key, v in mem.items()}
    t0 = time.perf_counter()
    R.calculate_advantages(full, cfg)
    t_gae = time.perf_counter() - t0
    t0 = time.perf_counter()
    R.train(agent, full, 0, max_minibatches=1)
    t_mb = time.perf_counter() - t0
    steps = args.epochs * (n * t // b)
    t_iter = t_roll + t_gae + t_mb * steps
    _progress(f"cpu baseline (cnn): rollout {k} steps {t_roll * k / t:.2f} s, minibatch {t_mb:.2f} s")
    return {"value": n * t / t_iter, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "torch": torch.__version__,
            "sample": (f"oracle/cnn_ref.py (torch-CPU Conv2d / Linear restatement; the reference has "
                       f"no pixel path), {threads} threads: {k} of {t} rollout steps + full GAE + 1 of "
                       f"{steps} minibatches of {b} at N={n}; extrapolated (rollout {t_roll:.2f}s, "
                       f"gae {t_gae:.3f}s, minibatch {t_mb:.2f}s)"),
            "seconds_per_iteration": t_iter}


def build(args, precision, env_kind, dev, rank):
    """(run, agent, helper, algo) for one leg of the workload (BASELINE configs[1] shapes)."""
    from mujoco_reinforcement_learning_amd.agent import make_agent
    from mujoco_reinforcement_learning_amd.algorithm import PPOEngine
    from mujoco_reinforcement_learning_amd.environments import (SyntheticVecEnvHelper,
                                                                make_synthetic_streams)
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    hidden = tuple(int(h) for h in args.hidden.split(","))
    n, t = args.num_envs, args.horizon
    run = make_run(num_envs=n, horizon=t, obs_dim=args.obs_dim, act_dim=args.act_dim,
                   window=args.window, hidden=hidden, batch_size=args.batch, epochs=args.epochs,
                   rng=args.rng, seed=rank, precision=precision,
                   rollout_graph=not args.no_graphs, train_graph=not args.no_graphs,
                   feature_extractor={"lstm": "LSTM", "cnn": "CNN"}.get(args.model, "MLP"),
                   latent=args.latent)
    torch.manual_seed(0)  # identical initial parameters on every rank
    agent = make_agent(run, device=dev)
    if args.model == "cnn":
        from mujoco_reinforcement_learning_amd.cnn import SyntheticPixelVecEnvHelper
        streams = make_synthetic_streams(n, t, 1, seed=1000 + rank, device=dev)
        helper = SyntheticPixelVecEnvHelper(streams, run, device=dev, seed=1000 + rank)
        return run, agent, helper, PPOEngine(helper, agent, log=lambda m: None)
    streams = make_synthetic_streams(n, t, args.obs_dim, seed=1000 + rank, device=dev)
    if env_kind == "host":
        from mujoco_reinforcement_learning_amd.environments import HostPhysicsVecEnvHelper
        helper = HostPhysicsVecEnvHelper(streams, run, device=dev, workers=args.env_workers)
    else:
        helper = SyntheticVecEnvHelper(streams, run, device=dev)
    algo = PPOEngine(helper, agent, log=lambda m: None)
    return run, agent, helper, algo


def time_iterations(algo, steps, warmup, world, dev) -> float:
    """W untimed iterations, then K timed ones bracketed by barrier + synchronize; the max over
    ranks of the wall time."""
    for _ in range(warmup):
        algo._iterate()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        algo._iterate()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(tt)
    return elapsed


def leg(args, precision, env_kind, dev) -> dict:
    """One extra single-GPU leg of the same workload (not `value`): its env-steps/s."""
    _progress(f"leg: precision {precision}, env {env_kind}")
    run, agent, helper, algo = build(args, precision, env_kind, dev, 0)
    try:
        elapsed = time_iterations(algo, args.leg_steps, 1, 1, dev)
    finally:
        if hasattr(helper, "close"):
            helper.close()
    n, t = args.num_envs, args.horizon
    return {"value": n * t * args.leg_steps / elapsed, "unit": "env-steps/s",
            "ms_per_step": 1000 * elapsed / args.leg_steps, "steps": args.leg_steps,
            "warmup": 1, "precision": precision,
            "env": ("device (synthetic dynamics on the GPU)" if env_kind == "device" else
                    f"host pool ({args.env_workers} worker processes in 2 groups, page-locked "
                    "device-mapped shared memory: obs / reward / terminated read and actions "
                    "written over PCIe every step, pipelined by ppo_host_rollout)")}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("for --gpus > 1 launch with torch.distributed.run (one rank per GPU)")
    # rehearsal knobs (not the measured configuration): PPO_BENCH_BACKEND=gloo and
    # PPO_BENCH_ONE_DEVICE=1 run N ranks on one GPU to exercise the data-parallel path
    if os.environ.get("PPO_BENCH_ONE_DEVICE") == "1":
        local = 0
        if world > 1:  # the in-launch fold needs its whole grid resident: not with N ranks per GPU
            os.environ.setdefault("PPO_FUSED_FOLD", "0")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("PPO_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group(backend)

    hidden = tuple(int(h) for h in args.hidden.split(","))
    n, t = args.num_envs, args.horizon
    run, agent, helper, algo = build(args, args.precision, args.env, dev, rank)
    elapsed = time_iterations(algo, args.steps, args.warmup, world, dev)
    if rank == 0:
        _progress(f"timed: {1000 * elapsed / args.steps:.2f} ms per iteration")
    classes, kernels = {}, {}
    if not args.no_timing:
        # Per-kernel durations: HIP event pairs on each dispatch packet, over --timing-iters
        # iterations of the same workload run right after the timed region with the hipGraphs
        # off (a replayed graph node cannot carry a per-dispatch event pair).
        ec = run.engine_config
        saved = (ec.rollout_graph, ec.train_graph)
        ec.rollout_graph, ec.train_graph = False, False
        agent.engine.timing(True, capacity=200000)
        for _ in range(args.timing_iters):
            algo._iterate()
        torch.cuda.synchronize()
        classes = agent.engine.timing_read()
        kernels = agent.engine.timing_kernels()
        agent.engine.timing(False)
        ec.rollout_graph, ec.train_graph = saved

    value = world * n * t * args.steps / elapsed
    metric = METRICS[args.model]
    if args.model == "mlp" and (args.obs_dim, args.act_dim, hidden, n) != (17, 6, (256, 256), 4096):
        # a non-headline MLP config (e.g. BASELINE configs[2] Ant, configs[3]'s Humanoid shard):
        # its own metric string, never the HalfCheetah headline's
        metric = (f"env-steps/sec {_ENV_NAMES.get((args.obs_dim, args.act_dim), 'custom')} "
                  f"{n} envs/GPU, {'x'.join(map(str, hidden))} MLP, {world}x MI355X")
    line = {"metric": metric, "value": value, "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (seeded device streams; action-dependent synthetic dynamics)",
            "config": {"workload": (f"{_ENV_NAMES.get((args.obs_dim, args.act_dim), 'custom')} "
                                    f"shapes: {n} envs/GPU x {t} steps, obs "
                                    f"{args.obs_dim}, act {args.act_dim}, actor+critic "
                                    + (f"BiLSTM(latent {args.latent}, window {args.window}) + "
                                       if args.model == "lstm" else "")
                                    + ("Nature-DQN CNN encoder (84x84x3 u8 frames -> 3136) + "
                                       if args.model == "cnn" else "")
                                    + f"{'x'.join(map(str, hidden))} ReLU MLP, PPO {args.epochs} "
                                    f"epochs x {n * t // args.batch} minibatches of {args.batch}"),
                       "num_envs_per_gpu": n, "horizon": t, "minibatch": args.batch,
                       "epochs": args.epochs, "rng": args.rng, "hipgraphs": not args.no_graphs,
                       "env": ("device (synthetic dynamics on the GPU)" if args.env == "device"
                               else f"host pool ({args.env_workers} worker processes, page-locked "
                                    "device-mapped shared memory, ppo_host_rollout)"),
                       "parallelism": (f"dp{world} (env-sharded, RCCL grad all-reduce)"
                                       if os.environ.get("PPO_DP_REHEARSE") != "1" or world > 1
                                       else "dp1 rehearsal (the data-parallel step sequence, "
                                            "no peer: PPO_DP_REHEARSE=1)")}}
    if kernels:
        traffic = load_traffic(args.traffic)
        name, c = max(kernels.items(), key=lambda kv: kv[1]["ms"])
        line["roofline"] = roofline(name, c, traffic)
        gae = {k: v for k, v in kernels.items() if v["class"] == "gae"}
        if gae:
            gname, gc = max(gae.items(), key=lambda kv: kv[1]["ms"])
            line["gae_roofline"] = roofline(gname, gc, traffic, force_hbm=True)
        ti = max(args.timing_iters, 1)
        line["kernel_classes_ms_per_step"] = {k: v["ms"] / ti for k, v in classes.items()
                                              if v["launches"]}
        line["kernels_ms_per_step"] = {k: round(v["ms"] / ti, 4) for k, v in
                                       sorted(kernels.items(), key=lambda kv: -kv[1]["ms"])}
    if world == 1 and not args.no_legs:
        del algo, agent
        torch.cuda.empty_cache()
        if args.precision != "f32":
            # the reference's precision on the same workload (f32 parity mode)
            line["f32_leg"] = leg(args, "f32", args.env, dev)
        if args.env != "host":
            # s8(d)'s t_iter includes the per-step obs H2D and action D2H: the host-pool env
            line["pcie_inclusive_leg"] = leg(args, args.precision, "host", dev)
    if rank == 0 and world == 1 and args.cpu_baseline:
        line["cpu_baseline"] = (cpu_baseline_cnn(args, hidden) if args.model == "cnn"
                                else cpu_baseline(args, hidden))
    if rank == 0:
        print(json.dumps(line), flush=True)
    if hasattr(helper, "close"):
        helper.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
