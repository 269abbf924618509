#!/bin/bash
# GPU tests + one bench line (no CPU baseline) -> gpurun_out/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_quick.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_quick.json").read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 2))
print("roofline", d["roofline"]["kernel"], round(d["roofline"]["frac"], 3), round(d["roofline"]["avg_launch_us"], 1))
for k, v in list(d["kernels_ms_per_step"].items())[:14]:
    print(f"  {v:8.3f}  {k}")
PY
