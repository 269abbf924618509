#!/bin/bash
# Fused bf16 update: its GPU tests, then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "bf16" > gpurun_out/fused_tests.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/fused_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/fused_tests.log | tail -12
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_fused.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_fused.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(round(d["value"]), round(d["ms_per_step"], 2), r["kernel"], r["bound"], round(r["frac"], 3), round(r["avg_launch_us"], 1))
for k, v in list(d["kernels_ms_per_step"].items())[:12]:
    print(f"   {v:8.3f}  {k}")
PY
