"""GAE scan bandwidth sweep over the number of envs (T = 128, f64 rewards, time-major buffers).

Algorithmic bytes per element: read V 4 + V' 4 + reward 8 + terminated 1, write adv 4 +
vtarget 4 = 25 B (done is derived from terminated in-kernel).  Prints one JSON line per N.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mujoco_reinforcement_learning_amd import engine as E  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    t = 128
    for n in (4096, 16384, 65536, 262144, 1048576):
        g = torch.Generator(device=dev).manual_seed(n)
        v = torch.randn(t, n, device=dev, generator=g)
        vn = torch.randn(t, n, device=dev, generator=g)
        r = torch.randn(t, n, device=dev, generator=g, dtype=torch.float64)
        term = torch.rand(t, n, device=dev, generator=g) < 0.01
        adv = torch.empty(t, n, device=dev)
        vt = torch.empty(t, n, device=dev)
        for _ in range(3):
            E.gae(v, vn, r, term, 0.99, 0.98, adv, vt)
        reps = 20
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            E.gae(v, vn, r, term, 0.99, 0.98, adv, vt)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / reps
        gbs = 25.0 * n * t / (us * 1e-6) / 1e9
        print(json.dumps({"kernel": "gae", "num_envs": n, "horizon": t, "avg_us": us,
                          "GBps": gbs, "frac_of_8TBps": gbs / 8000.0}), flush=True)


if __name__ == "__main__":
    main()
