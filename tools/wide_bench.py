"""Time the wide-path bf16 GEMMs at the Humanoid minibatch shapes (B = 65,536 rows, 3x512, O=376)
and, as a known-good ceiling on the same device, torch's bf16 matmul (hipBLASLt) of the same
shapes.  usage: python tools/wide_bench.py [iters]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mujoco_reinforcement_learning_amd import _lib  # noqa: E402

FWD, DGRAD, F32, WGRAD = 0, 1, 2, 3


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
    B = 65536
    out = []

    def timed(fn):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3  # us

    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)
    for name, kind, m, n, k, splits in [("fwd L1 512x512", FWD, B, 512, 512, 1),
                                        ("fwd L0 376->512", FWD, B, 512, 384, 1),
                                        ("dgrad 512x512", DGRAD, B, 512, 512, 1),
                                        ("wgrad 512x512", WGRAD, 512, 512, B, 16),
                                        ("wgrad L0 512x376", WGRAD, 512, 376, B, 16),
                                        ("head z f32", F32, B, 32, 512, 1),
                                        ("rollout fwd 1024", FWD, 1024, 512, 512, 1)]:
        if kind == WGRAD:
            a = r(B, 512)
            b = r(B, 384 if n == 376 else n)
            c = torch.empty(splits, m, n, device=dev)
            fn = lambda: _lib.check(lib.ppo_wide_gemm(kind, m, n, k, p(a), a.shape[1], p(b),
                                                      b.shape[1], p(c), n, None, None, None, 0,
                                                      splits, None, st))
            flops = 2.0 * m * n * k
            ref = lambda: torch.matmul(a[:, :m].t(), b[:, :n])
        else:
            a = r(m, k)
            b = r(n, k)
            c = (torch.empty(m, n, device=dev) if kind == F32 else r(m, n))
            aux = c.clone() if kind == DGRAD else None
            cs = torch.empty((m + 63) // 64, n, device=dev) if kind == DGRAD else None  # >= any row tile
            bias = torch.zeros(n, device=dev) if kind == FWD else None
            fn = lambda: _lib.check(lib.ppo_wide_gemm(kind, m, n, k, p(a), k, p(b), k, p(c), n,
                                                      p(bias), p(aux), p(cs), 0, 1, None, st))
            flops = 2.0 * m * n * k
            ref = lambda: torch.matmul(a, b.t())
        us_ref = timed(ref)
        for cfg in ("default", "1"):  # PPO_WIDE_CFG variants (wide_gemm.hip run_kind)
            if cfg == "default":
                os.environ.pop("PPO_WIDE_CFG", None)
            else:
                os.environ["PPO_WIDE_CFG"] = cfg
            us = timed(fn)
            rec = {"gemm": name, "cfg": cfg, "us": round(us, 2),
                   "tflops": round(flops / us / 1e6, 1),
                   "frac_bf16_peak": round(flops / us / 1e6 / 2516.6, 3),
                   "torch_hipblaslt_us": round(us_ref, 2),
                   "torch_tflops": round(flops / us_ref / 1e6, 1)}
            out.append(rec)
            print(json.dumps(rec), flush=True)
        os.environ.pop("PPO_WIDE_CFG", None)


if __name__ == "__main__":
    main()
