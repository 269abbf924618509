#!/bin/bash
# Full GPU test suite, then the default bench line (kernel table).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { echo TESTS FAILED; grep -E "PASS|FAIL|Error|error" gpurun_out/gpu_all.log | tail -15; tail -50 gpurun_out/gpu_all.log; exit 1; }
grep -cE "PASSED" gpurun_out/gpu_all.log; tail -1 gpurun_out/gpu_all.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_all.json 2> gpurun_out/bench_all.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_all.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_all.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(round(d["value"]), round(d["ms_per_step"], 2), r["kernel"], r["bound"], round(r["frac"], 3), round(r["avg_launch_us"], 1))
for k, v in list(d["kernels_ms_per_step"].items())[:14]:
    print(f"   {v:8.3f}  {k}")
PY
