"""The standalone GAE scan (ppo_gae -> gae_pipe_kernel) at the headline's 4096 envs and the sweep's
16384 / 65536, T = 128, f64 rewards: REPS back-to-back launches per size, for rocprofv3
--kernel-trace (per-dispatch durations by grid size: tools/gae_sizes.py --parse <kernel_trace.csv>)
next to the engine's per-dispatch HIP events (printed as JSON).  25 algorithmic bytes per
(env, step)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = (4096, 16384, 65536)
T = 128


def run(reps=200, kernels=("pipe", "chain")):
    import torch
    from mujoco_reinforcement_learning_amd import engine as E
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    dev = torch.device("cuda", 0)
    agent = PPOEngineAgent(make_run(hidden=(64, 64), num_envs=64), device=dev)  # a ctx for timing
    out = []
    for kernel in kernels:
        os.environ["PPO_GAE_KERNEL"] = kernel
        for n in SIZES:
            g = torch.Generator(device=dev).manual_seed(n)
            v = torch.randn(T, n, device=dev, generator=g)
            vn = torch.randn(T, n, device=dev, generator=g)
            r = torch.randn(T, n, device=dev, generator=g, dtype=torch.float64)
            term = torch.rand(T, n, device=dev, generator=g) < 0.01
            adv, vt = torch.empty(T, n, device=dev), torch.empty(T, n, device=dev)
            for _ in range(reps):  # untimed (rocprof sees them)
                E.gae(v, vn, r, term, 0.99, 0.98, adv, vt, force_last_done=True)
            torch.cuda.synchronize()
            agent.engine.timing(True, capacity=4 * reps)
            for _ in range(reps):
                E.gae(v, vn, r, term, 0.99, 0.98, adv, vt, force_last_done=True)
            torch.cuda.synchronize()
            ks = agent.engine.timing_kernels()
            agent.engine.timing(False)
            name, rec = max(ks.items(), key=lambda kv: kv[1]["ms"])
            us = 1e3 * rec["ms"] / rec["launches"]
            out.append({"kernel": name, "num_envs": n, "horizon": T, "events_avg_us": us,
                        "events_frac_hbm": 25.0 * n * T / (us * 1e-6) / 8e12})
    print(json.dumps(out))


def parse(path):
    """Per-dispatch rocprofv3 durations of the GAE scan kernels grouped by kernel and grid size."""
    import csv
    import collections
    d = collections.defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if "gae_pipe_kernel" not in name and "gae_chain_kernel" not in name:
                continue
            kind = "chain" if "chain" in name else "pipe"
            d[(kind, int(row["Grid_Size_X"]))].append(
                int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    out = []
    for (kind, grid), v in sorted(d.items()):
        v.sort()
        # grid threads = blocks x (EB * 16 [+ 64: the chain wave]), EB = 16 or 32 envs per block
        n = next(x for x in SIZES for eb in (16, 32)
                 if (x // eb) * (eb * 16 + (64 if kind == "chain" else 0)) == grid)
        o = {"kernel": kind, "num_envs": n, "grid_threads": grid, "dispatches": len(v),
             "mean_us": sum(v) / len(v) / 1e3, "median_us": v[len(v) // 2] / 1e3,
             "p10_us": v[len(v) // 10] / 1e3}
        o["median_frac_hbm"] = 25.0 * n * T / (o["median_us"] * 1e-6) / 8e12
        o["mean_frac_hbm"] = 25.0 * n * T / (o["mean_us"] * 1e-6) / 8e12
        out.append(o)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
    else:
        run()
