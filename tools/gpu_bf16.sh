#!/bin/bash
# bf16-mode GPU tests + bf16 and f32 bench lines -> gpurun_out/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "bf16 or graph or minibatch" > gpurun_out/bf16_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/bf16_tests.log; exit 1; }
tail -2 gpurun_out/bf16_tests.log
for prec in bf16 f32; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --precision $prec > gpurun_out/bench_$prec.json 2> gpurun_out/bench_$prec.err || { echo BENCH $prec FAILED; tail -20 gpurun_out/bench_$prec.err; exit 1; }
  python - $prec <<'PY'
import json, sys
p = sys.argv[1]
d = json.loads(open(f"gpurun_out/bench_{p}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(p, round(d["value"]), round(d["ms_per_step"], 2), r["kernel"], r["bound"], round(r["frac"], 3))
for k, v in list(d["kernels_ms_per_step"].items())[:9]:
    print(f"   {v:8.3f}  {k}")
PY
done
