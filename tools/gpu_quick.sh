#!/bin/bash
# Targeted GPU tests (K = pytest -k expression), then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "${K:-staged or graphs or bf16}" > gpurun_out/gpu_quick.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/gpu_quick.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/gpu_quick.log | tail -20
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_q.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_q.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(round(d["value"]), round(d["ms_per_step"], 2), r["kernel"], r["bound"], round(r["frac"], 3), round(r["avg_launch_us"], 1))
for k, v in list(d["kernels_ms_per_step"].items())[:12]:
    print(f"   {v:8.3f}  {k}")
PY
