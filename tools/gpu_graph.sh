#!/bin/bash
# Graph-vs-eager parity tests, then the bench with and without hipGraph replay.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_iteration.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_graph.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/gpu_graph.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/gpu_graph.log | tail -12
for mode in "" "--no-graphs"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $mode > gpurun_out/bench_g.json 2> gpurun_out/bench_g.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_g.err; exit 1; }
  python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_g.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(d["config"]["hipgraphs"], round(d["value"]), round(d["ms_per_step"], 2), r["kernel"], r["bound"], round(r["frac"], 3), round(r["avg_launch_us"], 1))
for k, v in list(d["kernels_ms_per_step"].items())[:10]:
    print(f"   {v:8.3f}  {k}")
PY
done
