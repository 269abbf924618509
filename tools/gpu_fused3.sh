#!/bin/bash
# Fused-kernel GPU tests (bf16 emulation, staged, graphs, determinism), phase stamps, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "bf16 or staged or graphs or fused" > gpurun_out/fused3.log 2>&1 || { echo TESTS FAILED; grep -E "PASSED|FAILED" gpurun_out/fused3.log | tail; tail -40 gpurun_out/fused3.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/fused3.log | tail -20
timeout -k 10 200 python tools/fused_phases.py || { echo PHASES FAILED; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_f3.json 2> gpurun_out/bench_f3.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_f3.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_f3.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(round(d["value"]), round(d["ms_per_step"], 2), r["kernel"], r["bound"], round(r["frac"], 3), round(r["avg_launch_us"], 1))
for k, v in list(d["kernels_ms_per_step"].items())[:12]:
    print(f"   {v:8.3f}  {k}")
PY
