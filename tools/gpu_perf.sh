#!/bin/bash
# Perf check of the fused kernels: phase stamps, then the default bench line (no tests).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python tools/fused_phases.py || { echo PHASES FAILED; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_p.json 2> gpurun_out/bench_p.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_p.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_p.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(round(d["value"]), round(d["ms_per_step"], 2), r["kernel"], r["bound"], round(r["frac"], 3), round(r["avg_launch_us"], 1))
for k, v in list(d["kernels_ms_per_step"].items())[:8]:
    print(f"   {v:8.3f}  {k}")
PY
