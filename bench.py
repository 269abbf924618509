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
                bench_traffic.json when present (same command under rocprofv3 --pmc)
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
    p.add_argument("--traffic", default=os.path.join(ROOT, "bench_traffic.json"),
                   help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py output)")
    p.add_argument("--gae-sweep", default="4096,16384,65536",
                   help="env counts at which the headline line also times the standalone GAE scan "
                        "(the headline's 4096 and its bandwidth ceiling beyond; empty for none)")
    p.add_argument("--legs", default="ant,humanoid,cnn,lstm",
                   help="BASELINE-config legs the default N=1 line carries (comma list of ant, "
                        "humanoid, cnn, lstm; empty for none)")
    args = p.parse_args()
    apply_model_defaults(args, p.get_default)
    return args


MODEL_DEFAULTS = {
    "lstm": {"num_envs": 1024, "obs_dim": 348, "act_dim": 17, "hidden": "256,256,128,128",
             "batch": 16384, "window": 5},
    "cnn": {"num_envs": 1024, "obs_dim": 84 * 84 * 3, "act_dim": 6, "batch": 16384},
}


def apply_model_defaults(args, default_of) -> None:
    """The --model lstm / cnn workloads' shapes where the command line left the MLP defaults."""
    for k, v in MODEL_DEFAULTS.get(args.model, {}).items():
        if getattr(args, k) == default_of(k):
            setattr(args, k, v)
    if args.model == "lstm":
        args.no_legs = True
        args.cpu_baseline = False
    if args.model == "cnn":
        args.no_legs = True
    if args.window is None:
        args.window = 1


def load_traffic(path, workload=None):
    """{kernel name: HBM bytes per launch} from PMC passes over the same workload
    (tools/pmc_traffic.py; FETCH_SIZE x2 + WRITE_SIZE per MI355X_MICROARCH.md), or {}.  The table
    holds one sub-table per workload (tools/merge_traffic.py): the headline's at the top level and
    each leg's under by_workload[name] -- the layered GEMM instantiations are shared by the pixel
    and BiLSTM heads with different shapes, so a leg only ever reads its own workload's bytes."""
    if not path or not os.path.exists(path):
        return {}
    with open(path) as f:
        t = json.load(f)
    if workload is None:
        return t.get("bytes_per_launch", {})
    return t.get("by_workload", {}).get(workload, {})


def traffic_workload(args):
    """The traffic sub-table of a run: None for the headline, else the config leg it measures."""
    if args.model in ("cnn", "lstm"):
        return args.model
    return {(27, 8): "ant", (376, 17): "humanoid"}.get((args.obs_dim, args.act_dim))


# gymnasium observation / action sizes of the BASELINE configs (SURVEY.md s8 notation)
_ENV_NAMES = {(17, 6): "HalfCheetah-v4", (27, 8): "Ant-v4", (376, 17): "Humanoid-v4",
              (348, 17): "main.py humanoid (O=348)", (84 * 84 * 3, 6): "cheetah-run pixels"}


def _traffic_of(traffic, name):
    """PMC bytes per launch of ``name``; a fused-update name carries its phase schedule as the last
    template argument (PPO_FUSED_SCHED: an LDS-level reordering, the same global loads and stores),
    so a table measured under another schedule of the same instantiation is used for it."""
    if name in traffic:
        return traffic[name]
    import re
    base = re.sub(r", \d+>$", ">", name)
    if name.startswith("fused_update_kernel<"):
        for k, v in traffic.items():
            if k == base or re.sub(r", \d+>$", ">", k) == base:
                return v
    return None


def roofline(name, c, traffic, force_hbm=False):
    """Roofline of one kernel instantiation from its live event records.  The bound is the roof
    the kernel's own algorithmic work hits first: MFMA (FLOPs / dense peak of its dtype) or HBM
    (bytes / 8 TB/s); achieved = that work per launch / mean launch duration."""
    launches = max(c["launches"], 1)
    avg_s = c["ms"] * 1e-3 / launches
    # the fused update kernel, the wide path's GEMMs (wide_gemm / wide_pair) and the pixel encoder's LDS-staged
    # convolutions (conv_pixel.h, conv_lds.h) are bf16-only; the layered GEMMs and conv_kernel
    # carry their dtype in the name
    bf16 = ("bf16" in name or name.startswith("wide_") or c["class"] == "fused_update"
            or "_lds_kernel" in name or name.startswith("pixel_"))
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
            "traffic": _traffic_of(traffic, name), "avg_launch_us": avg_s * 1e6,
            "launches": c["launches"],
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
        elapsed = time_iterations(algo, args.leg_steps, 2, 1, dev)  # eager, then graph capture
    finally:
        if hasattr(helper, "close"):
            helper.close()
    n, t = args.num_envs, args.horizon
    return {"value": n * t * args.leg_steps / elapsed, "unit": "env-steps/s",
            "ms_per_step": 1000 * elapsed / args.leg_steps, "steps": args.leg_steps,
            "warmup": 2, "precision": precision,
            "env": ("device (synthetic dynamics on the GPU)" if env_kind == "device" else
                    f"host pool ({args.env_workers} worker processes in 2 groups, page-locked "
                    "device-mapped shared memory: obs / reward / terminated read and actions "
                    "written over PCIe every step, pipelined by ppo_host_rollout)")}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, timeout: float = None) -> int:
    """``bench.py --gpus N`` started as one plain process: start N rank processes of this same
    command (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their env,
    as torch.distributed.run would set them), forward rank 0's JSON line, and return non-zero if
    any rank fails.  This parent never touches the GPU (no HIP call before or after the
    children start), and when one rank dies the others are terminated by their own PIDs rather
    than left waiting in a collective.

    Wall-clock bound (PPO_BENCH_RANK_TIMEOUT seconds, default 1200): a rank blocked inside a
    collective never exits on its own, so on expiry every rank still alive is terminated (then
    killed), ONE JSON line with ``error`` and the ranks still alive is printed, and the exit
    status is 124.  Nothing is re-executed."""
    import subprocess
    if timeout is None:
        timeout = float(os.environ.get("PPO_BENCH_RANK_TIMEOUT", "1200"))
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                                      env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr))
    import threading
    chunks = []
    reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    rcs = [None] * n
    deadline = time.monotonic() + timeout
    timed_out = None
    # reap in completion order; after the first failure terminate the rest
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
                if rcs[i] not in (None, 0):
                    for q in procs:
                        if q.poll() is None:
                            q.terminate()
        if timed_out is None and time.monotonic() > deadline and any(rc is None for rc in rcs):
            timed_out = [i for i, rc in enumerate(rcs) if rc is None]
            _progress(f"ranks {timed_out} still running after {timeout:.0f} s: terminating them")
            for i in timed_out:
                procs[i].terminate()
            for i in timed_out:
                try:
                    procs[i].wait(timeout=10)
                except subprocess.TimeoutExpired:
                    procs[i].kill()
                    procs[i].wait()
                rcs[i] = procs[i].returncode
        time.sleep(0.05)
    reader.join(timeout=10)
    # rank 0's JSON line to stdout; library chatter (e.g. gloo's connection lines) to stderr
    out = b"".join(chunks).decode(errors="replace").splitlines()
    if timed_out is not None:
        for ln in out:
            print(ln, file=sys.stderr)
        print(json.dumps({"metric": METRIC, "value": None, "unit": "env-steps/s", "n_gpus": n,
                          "error": f"rank processes still running after {timeout:.0f} s "
                                   f"(PPO_BENCH_RANK_TIMEOUT); terminated",
                          "alive_ranks": timed_out, "exit_codes": rcs}), flush=True)
        return 124
    for ln in out:
        print(ln, file=sys.stdout if ln.startswith("{") else sys.stderr)
    sys.stdout.flush()
    bad = [(i, rc) for i, rc in enumerate(rcs) if rc != 0]
    if bad:
        _progress(f"rank(s) failed: {bad}")
        return 1
    return 0


def launch_check(args, world, rank) -> None:
    """PPO_BENCH_LAUNCH_CHECK=1 (CPU tests of the launcher): the rank plumbing of main() -- gloo
    rendezvous, barrier-bracketed timing, max over ranks, rank 0's JSON line -- with no GPU work.
    PPO_BENCH_LAUNCH_CHECK_FAIL_RANK=r makes rank r exit with status 3 before the rendezvous (the
    launcher must then stop the other ranks and fail); PPO_BENCH_LAUNCH_CHECK_HANG_RANK=r makes
    rank r block after the rendezvous, so the others wait in the next collective (the launcher's
    wall-clock bound must end the run); PPO_BENCH_LAUNCH_CHECK_CAPTURE_FAIL_RANK=r runs the
    update-loop capture agreement (DataParallel.capture_agreed) with a stand-in communicator whose
    capture fails on rank r only, then the exchanges of the eager fallback, and reports the
    resulting ``comm`` and whether the ranks' results agree bitwise."""
    from mujoco_reinforcement_learning_amd.distributed import DataParallel
    if os.environ.get("PPO_BENCH_LAUNCH_CHECK_FAIL_RANK") == str(rank):
        sys.exit(3)
    torch.distributed.init_process_group("gloo")
    t0 = time.perf_counter()
    torch.distributed.barrier()
    if os.environ.get("PPO_BENCH_LAUNCH_CHECK_HANG_RANK") == str(rank):
        while True:
            time.sleep(1)
    tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
    line = {"metric": METRIC, "value": None, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "launch_check": True}
    fail_rank = os.environ.get("PPO_BENCH_LAUNCH_CHECK_CAPTURE_FAIL_RANK")
    if fail_rank is not None:
        dp = DataParallel()

        class _StandIn:  # the native communicator's interface over the gloo group
            retired = False

            def retire(self):
                self.retired = True

            def allreduce(self, t):
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM)

        comm = dp.comm = _StandIn()

        def capture():
            if str(rank) == fail_rank:
                raise RuntimeError(f"operation not permitted when stream is capturing (rank {rank})")

        reason = dp.capture_agreed(capture)
        # the eager fallback's exchanges: three all-reduces of rank-dependent gradients
        g = torch.arange(8, dtype=torch.float32) * (rank + 1) / 7.0
        for _ in range(3):
            dp.allreduce_grad(g)
            g.mul_(0.5)
        gathered = [torch.empty_like(g) for _ in range(world)]
        torch.distributed.all_gather(gathered, g)
        line["capture"] = {"fallback": reason is not None, "reason": reason,
                           "native_retired": comm.retired,
                           "replicas_bitwise_equal": all(torch.equal(gathered[0], x)
                                                         for x in gathered)}
        line["comm"] = dp.comm_info()
    if rank == 0:
        print(json.dumps(line), flush=True)
    torch.distributed.destroy_process_group()


def _macs_per_row(agent) -> int:
    """Forward multiply-accumulates per row of both nets, counted from the modules: Linear
    in*out; LSTM per layer and direction W * 4H * (in + H) over the window (the recurrent GEMMs
    run once per window slot)."""
    window = agent.run.environment_config.window_length
    macs = 0
    for m in agent.networks.modules():
        if isinstance(m, torch.nn.Linear):
            macs += m.in_features * m.out_features
        elif isinstance(m, torch.nn.LSTM):
            dirs = 2 if m.bidirectional else 1
            for layer in range(m.num_layers):
                inp = m.input_size if layer == 0 else m.hidden_size * dirs
                macs += dirs * window * 4 * m.hidden_size * (inp + m.hidden_size)
    return macs


# BASELINE.json configs carried as legs of the default line (their own metric strings)
CONFIG_LEGS = {
    "ant": dict(model="mlp", num_envs=4096, obs_dim=27, act_dim=8, hidden="256,256", batch=65536,
                window=1, baseline="configs[2] Ant-v4, 4096 envs, 2x256 MLP, 1x MI355X"),
    # configs[3]: 8192 envs over 8 GPUs = 1024 envs per rank; global minibatch 65,536 = 8 ranks x
    # B_local 8,192, i.e. 16 minibatches per epoch (local data parallelism divides each rank's
    # loss by B_local * world, so the all-reduced gradient is the global-minibatch mean)
    "humanoid": dict(model="mlp", num_envs=1024, obs_dim=376, act_dim=17, hidden="512,512,512",
                     batch=8192, window=1,
                     baseline="configs[3] Humanoid-v4, 8192 envs, 3x512 MLP, 8x MI355X env-sharded: "
                              "one rank's shard (1024 envs, B_local 8192 of the global 65,536)"),
    "cnn": dict(model="cnn", baseline="configs[4] dm_control cheetah-run 84x84x3 pixels, 1024 "
                                      "envs, Nature-DQN CNN encoder, 1x MI355X"),
    "lstm": dict(model="lstm", baseline="the reference PPOAgent's BiLSTM actor-critic on main.py's "
                                        "network (O=348, W=5, latent 256, [256,256,128,128], A=17), "
                                        "1024 envs, 1x MI355X"),
}


def config_leg(args, name, dev, steps=None, **over) -> dict:
    """One BASELINE-config leg on this GPU: its own workload, metric string, ms_per_step and
    roofline (the leg's dominant kernel from live events; the whole iteration's algorithmic FLOPs
    against the bf16 peak only if an engine recorded no per-kernel events)."""
    spec = dict(CONFIG_LEGS[name], **over)
    baseline = spec.pop("baseline")
    ns = argparse.Namespace(**vars(args))
    ns.model = spec.pop("model")
    for k in ("num_envs", "obs_dim", "act_dim", "hidden", "batch", "window", "horizon", "epochs"):
        setattr(ns, k, parse_defaults[k])
    ns.window, ns.no_timing = None, False
    for k, v in spec.items():
        setattr(ns, k, v)
    apply_model_defaults(ns, parse_defaults.get)
    steps = steps or args.leg_steps
    _progress(f"leg {name}: {ns.num_envs} envs, obs {ns.obs_dim}, act {ns.act_dim}, "
              f"hidden {ns.hidden}, B {ns.batch}, model {ns.model}")
    run, agent, helper, algo = build(ns, ns.precision, "device", dev, 0)
    try:
        elapsed = time_iterations(algo, steps, 2, 1, dev)  # warm-up 2: eager, then graph capture
        kernels = {}
        if hasattr(agent.engine, "timing"):
            ec = run.engine_config
            ec.rollout_graph, ec.train_graph = False, False
            agent.engine.timing(True, capacity=400000)
            algo._iterate()
            torch.cuda.synchronize()
            kernels = agent.engine.timing_kernels()
            agent.engine.timing(False)
        macs = _macs_per_row(agent)
    finally:
        if hasattr(helper, "close"):
            helper.close()
    n, t = ns.num_envs, ns.horizon
    hidden = tuple(int(h) for h in ns.hidden.split(","))
    out = {"metric": leg_metric(ns, hidden, 1), "baseline_config": baseline,
           "value": n * t * steps / elapsed, "unit": "env-steps/s",
           "ms_per_step": 1000 * elapsed / steps, "steps": steps, "warmup": 2,
           "dtype": ns.precision, "workload": workload(ns, hidden),
           "minibatches_per_epoch": n * t // ns.batch}
    flop_step = (2 + 6 * ns.epochs) * macs  # 2F rollout + E x 3 x 2F update
    e2e = flop_step * n * t * steps / elapsed / 1e12
    out["end_to_end"] = {"flop_per_env_step": flop_step, "achieved": e2e, "unit": "TFLOP/s",
                         "peak": PEAK_BF16_MFMA_TFLOPS, "frac": e2e / PEAK_BF16_MFMA_TFLOPS}
    if kernels:
        kname, c = max(kernels.items(), key=lambda kv: kv[1]["ms"])
        # a leg run with overridden shapes has no table of its own (traffic null)
        out["roofline"] = roofline(kname, c, load_traffic(args.traffic, name if not over else f"{name}*"))
        out["kernels_ms_per_step"] = {k: round(v["ms"], 4) for k, v in
                                      sorted(kernels.items(), key=lambda kv: -kv[1]["ms"])[:8]}
    else:
        out["roofline"] = dict(out["end_to_end"], bound="mfma", kernel="whole iteration (no "
                               "per-kernel events in this context)", traffic=None)
    del algo, agent, helper, run
    torch.cuda.empty_cache()
    return out


def leg_metric(ns, hidden, world) -> str:
    if ns.model in ("lstm", "cnn"):
        return METRICS[ns.model]
    return (f"env-steps/sec {_ENV_NAMES.get((ns.obs_dim, ns.act_dim), 'custom')} "
            f"{ns.num_envs} envs/GPU, {'x'.join(map(str, hidden))} MLP, {world}x MI355X")


def workload(ns, hidden) -> str:
    n, t = ns.num_envs, ns.horizon
    return (f"{_ENV_NAMES.get((ns.obs_dim, ns.act_dim), 'custom')} shapes: {n} envs/GPU x {t} "
            f"steps, obs {ns.obs_dim}, act {ns.act_dim}, actor+critic "
            + (f"BiLSTM(latent {ns.latent}, window {ns.window}) + " if ns.model == "lstm" else "")
            + ("Nature-DQN CNN encoder (84x84x3 u8 frames -> 3136) + " if ns.model == "cnn" else "")
            + f"{'x'.join(map(str, hidden))} ReLU MLP, PPO {ns.epochs} epochs x "
            f"{n * t // ns.batch} minibatches of {ns.batch}")


parse_defaults = {"num_envs": 4096, "obs_dim": 17, "act_dim": 6, "hidden": "256,256",
                  "batch": 65536, "window": None, "horizon": 128, "epochs": 10}


def parallelism_label(world: int) -> str:
    rehearse = os.environ.get("PPO_DP_REHEARSE", "") if world == 1 else ""
    if rehearse == "1":
        return "dp1 rehearsal (the data-parallel step sequence, no peer: PPO_DP_REHEARSE=1)"
    if rehearse == "rccl":
        return ("dp1 rehearsal (the data-parallel step sequence with the native RCCL all-reduce "
                "of a world-1 communicator, graph-captured: PPO_DP_REHEARSE=rccl)")
    return f"dp{world} (env-sharded, RCCL grad all-reduce)"


def gae_sweep_points(agent, dev, t: int, ns) -> list:
    """ppo_gae (gae_pipe_kernel) alone at larger env counts, T steps, f64 rewards: 25 algorithmic
    bytes per (env, step) (V, V', reward, terminated in; adv, target out), kernel time from the
    engine's per-dispatch events (tools/gae_sweep.py's method)."""
    from mujoco_reinforcement_learning_amd import engine as E
    out = []
    for n in ns:
        g = torch.Generator(device=dev).manual_seed(n)
        v = torch.randn(t, n, device=dev, generator=g)
        vn = torch.randn(t, n, device=dev, generator=g)
        r = torch.randn(t, n, device=dev, generator=g, dtype=torch.float64)
        term = torch.rand(t, n, device=dev, generator=g) < 0.01
        adv, vt = torch.empty(t, n, device=dev), torch.empty(t, n, device=dev)
        for _ in range(3):
            E.gae(v, vn, r, term, 0.99, 0.98, adv, vt, force_last_done=True)
        torch.cuda.synchronize()
        agent.engine.timing(True, capacity=64)
        for _ in range(20):
            E.gae(v, vn, r, term, 0.99, 0.98, adv, vt, force_last_done=True)
        torch.cuda.synchronize()
        ks = agent.engine.timing_kernels()
        agent.engine.timing(False)
        name, rec = max(ks.items(), key=lambda kv: kv[1]["ms"])
        us = 1e3 * rec["ms"] / rec["launches"]
        gbs = 25.0 * n * t / (us * 1e-6) / 1e9
        out.append({"kernel": name, "num_envs": n, "horizon": t, "avg_launch_us": us,
                    "achieved": gbs, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
                    "algorithmic_per_launch": 25.0 * n * t})
        del v, vn, r, term, adv, vt
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if os.environ.get("PPO_BENCH_LAUNCH_CHECK") == "1":
        return launch_check(args, world, rank)
    # rehearsal knobs (not the measured configuration): PPO_BENCH_BACKEND=gloo and
    # PPO_BENCH_ONE_DEVICE=1 run N ranks on one GPU to exercise the data-parallel path
    if os.environ.get("PPO_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world == 1 and os.environ.get("PPO_DP_REHEARSE") == "rccl":
        # the data-parallel step sequence with the native RCCL all-reduce, graph-captured, on one
        # rank (DataParallel): a world-1 RCCL process group
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        torch.distributed.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
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
    comm = None
    if hasattr(algo, "dp"):
        # the exchange as it ran: the native communicator's own rank count (ppo_comm_query), the
        # process group's backend, and whether the update loop was replayed as one hipGraph
        comm = dict(algo.dp.comm_info(),
                    graph_captured=getattr(algo, "_tg_graph", None) is not None,
                    capture_failed=bool(getattr(algo, "_tg_capture_failed", False)))
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
        metric = leg_metric(args, hidden, world)
    line = {"metric": metric, "value": value, "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (seeded device streams; action-dependent synthetic dynamics)",
            "config": {"workload": workload(args, hidden),
                       "num_envs_per_gpu": n, "horizon": t, "minibatch": args.batch,
                       "epochs": args.epochs, "rng": args.rng, "hipgraphs": not args.no_graphs,
                       "env": ("device (synthetic dynamics on the GPU)" if args.env == "device"
                               else f"host pool ({args.env_workers} worker processes, page-locked "
                                    "device-mapped shared memory, ppo_host_rollout)"),
                       "parallelism": parallelism_label(world)},
            "comm": comm}
    if kernels:
        traffic = load_traffic(args.traffic, traffic_workload(args))
        name, c = max(kernels.items(), key=lambda kv: kv[1]["ms"])
        line["roofline"] = roofline(name, c, traffic)
        gae = {k: v for k, v in kernels.items() if v["class"] == "gae"}
        if gae:
            gname, gc = max(gae.items(), key=lambda kv: kv[1]["ms"])
            gr = roofline(gname, gc, traffic, force_hbm=True)
            if "records" in gname:
                # the fused scan + record pass counts every byte it moves, including the padding
                # of the 128-B row records; the payload-only figure drops that padding
                rows = n * t
                payload = 2 * args.window * args.obs_dim + 4 * args.act_dim + 12
                pb = gr["algorithmic_per_launch"] - (128 - payload) * rows
                # the headline figure counts the record's payload only; the
                # padded figure (every byte of the 128-B record written) stays as a secondary
                gr["with_record_padding"] = {
                    "achieved": gr["achieved"], "frac": gr["frac"],
                    "algorithmic_per_launch": gr["algorithmic_per_launch"],
                    "bytes_counted": "as below, but the full 128-B record written per (env, step)"}
                gr["achieved"] = pb / (gr["avg_launch_us"] * 1e-6) / 1e9
                gr["frac"] = gr["achieved"] / PEAK_HBM_GBS
                gr["algorithmic_per_launch"] = pb
                gr["bytes_counted"] = (f"reads: reward f64, V, V', terminated (scan, 25 B) + "
                                       f"state f32 {4 * args.window * args.obs_dim} B + actions "
                                       f"{4 * args.act_dim} B + old log-prob 4 B; writes: adv / "
                                       f"target 8 B + the record's {payload}-B payload (bf16 "
                                       f"state, actions, old log-prob, adv, target) per (env, step)")
            if args.gae_sweep and args.model == "mlp":
                # the standalone scan's bandwidth ceiling beyond the headline's 4096 envs
                gr["scan_sweep"] = gae_sweep_points(agent, dev, args.horizon,
                                                    [int(x) for x in args.gae_sweep.split(",")])
            line["gae_roofline"] = gr
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
        if args.model == "mlp" and (args.obs_dim, args.act_dim, hidden, n) == (17, 6, (256, 256),
                                                                                4096):
            for name in [x for x in args.legs.split(",") if x]:
                line[f"{name}_leg"] = config_leg(args, name, dev)
                if name == "humanoid":
                    # the same shard with one rank's B = 65,536 (2 minibatches per epoch): the
                    # round-3 measurement's setting, fewer and larger optimizer steps
                    line["humanoid_leg"]["b65536"] = {
                        k: v for k, v in config_leg(args, name, dev, batch=65536).items()
                        if k in ("value", "ms_per_step", "minibatches_per_epoch", "roofline")}
    if rank == 0 and world == 1 and args.cpu_baseline:
        line["cpu_baseline"] = (cpu_baseline_cnn(args, hidden) if args.model == "cnn"
                                else cpu_baseline(args, hidden))
    if rank == 0:
        print(json.dumps(line), flush=True)
    if hasattr(helper, "close"):
        helper.close()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
