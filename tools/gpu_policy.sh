#!/bin/bash
# Policy-step change check: fused observe/act + determinism + graph tests, then the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "observe or deterministic or graphs or smoke or iteration" > gpurun_out/policy_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error" gpurun_out/policy_tests.log | tail -15; tail -40 gpurun_out/policy_tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/policy_tests.log; tail -1 gpurun_out/policy_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_policy.json 2> gpurun_out/bench_policy.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_policy.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_policy.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(round(d["value"]), round(d["ms_per_step"], 2), r["kernel"], r["bound"], round(r["frac"], 3), round(r["avg_launch_us"], 1))
for k, v in list(d["kernels_ms_per_step"].items())[:14]:
    print(f"   {v:8.3f}  {k}")
PY
