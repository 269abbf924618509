"""Library GEMM ceiling at the update shapes (M = 65,536 rows, 256 x 256 layer): torch.mm
(hipBLASLt / rocBLAS) in f32, f32 with TF32/xf32 allowed, and bf16.  Prints TFLOP/s."""
import json
import torch


def bench(fn, reps=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    dev = torch.device("cuda", 0)
    m, k, n = 65536, 256, 256
    for dt in (torch.float32, torch.bfloat16):
        for tf32 in ((False, True) if dt == torch.float32 else (False,)):
            torch.backends.cuda.matmul.allow_tf32 = tf32
            a = torch.randn(m, k, device=dev, dtype=dt)
            w = torch.randn(n, k, device=dev, dtype=dt)
            g = torch.randn(m, n, device=dev, dtype=dt)
            for name, fn in (("fwd x@W^T", lambda: a @ w.t()),
                             ("dgrad g@W", lambda: g @ w),
                             ("wgrad g^T@x", lambda: g.t() @ a)):
                t = bench(fn)
                print(json.dumps({"dtype": str(dt), "tf32": tf32, "op": name,
                                  "us": t * 1e6, "tflops": 2 * m * n * k / t / 1e12}), flush=True)


if __name__ == "__main__":
    main()
