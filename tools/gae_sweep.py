"""GAE scan bandwidth sweep over the number of envs (T from $GAE_T, default 128; f64 rewards,
time-major buffers).

Kernel time comes from the engine's per-dispatch event pairs (a context's timing records the
ctx-free ppo_gae launches while it is on), not from events around a loop of Python calls: at
small N a back-to-back loop measures the host's dispatch rate (~9 us per call), not the kernel.
Algorithmic bytes per element: read V 4 + V' 4 + reward 8 + terminated 1, write adv 4 +
vtarget 4 = 25 B (done is derived from terminated in-kernel).  Prints one JSON line per N.
Usage: python tools/gae_sweep.py [N ...]   (PPO_GAE_KERNEL / PPO_GAE_EB select variants)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mujoco_reinforcement_learning_amd import engine as E  # noqa: E402


def main():
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    dev = torch.device("cuda", 0)
    t = int(os.environ.get("GAE_T", "128"))
    ctx = PPOEngineAgent(make_run(num_envs=64, hidden=(64, 64)), device=dev).engine
    ns = [int(a) for a in sys.argv[1:]] or [4096, 16384, 65536, 262144, 1048576]
    for n in ns:
        g = torch.Generator(device=dev).manual_seed(n)
        v = torch.randn(t, n, device=dev, generator=g)
        vn = torch.randn(t, n, device=dev, generator=g)
        r = torch.randn(t, n, device=dev, generator=g, dtype=torch.float64)
        term = torch.rand(t, n, device=dev, generator=g) < 0.01
        adv = torch.empty(t, n, device=dev)
        vt = torch.empty(t, n, device=dev)
        for _ in range(3):
            E.gae(v, vn, r, term, 0.99, 0.98, adv, vt)
        torch.cuda.synchronize()
        reps = 20
        ctx.timing(True, capacity=64)
        for _ in range(reps):
            E.gae(v, vn, r, term, 0.99, 0.98, adv, vt)
        torch.cuda.synchronize()
        ks = ctx.timing_kernels()
        ctx.timing(False)
        for name, rec in ks.items():
            us = 1e3 * rec["ms"] / rec["launches"]
            gbs = 25.0 * n * t / (us * 1e-6) / 1e9
            print(json.dumps({"kernel": name, "eb": os.environ.get("PPO_GAE_EB", "auto"),
                              "num_envs": n, "horizon": t, "avg_us": us, "GBps": gbs,
                              "frac_of_8TBps": gbs / 8000.0}), flush=True)


if __name__ == "__main__":
    main()
