#!/bin/bash
# One GPU call: GPU tests, the default (bf16) and f32 bench lines, rocprofv3 kernel-trace stats over
# the bench command, FETCH_SIZE / WRITE_SIZE PMC passes -> traffic per launch, timing agreement.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo GPU TESTS FAILED; tail -40 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
  tail -3 gpurun_out/gpu_tests_${TAG}.log
fi
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 300 python bench.py --precision f32 --no-cpu-baseline > gpurun_out/bench_${TAG}_f32.json 2> gpurun_out/bench_${TAG}_f32.err || { echo BENCH F32 FAILED; tail -20 gpurun_out/bench_${TAG}_f32.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_${TAG}_trace -o bench --output-format csv \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rp_${TAG}_bench.json 2> gpurun_out/rp_${TAG}_trace.log || { echo TRACE FAILED; tail -20 gpurun_out/rp_${TAG}_trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/rp_${TAG}_fetch -o fetch --output-format csv \
  -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-timing > gpurun_out/rp_${TAG}_fetch.log 2>&1 || { echo FETCH FAILED; tail -20 gpurun_out/rp_${TAG}_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/rp_${TAG}_write -o write --output-format csv \
  -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-timing > gpurun_out/rp_${TAG}_write.log 2>&1 || { echo WRITE FAILED; tail -20 gpurun_out/rp_${TAG}_write.log; exit 1; }
python tools/pmc_traffic.py $(find gpurun_out/rp_${TAG}_fetch -name "*counter_collection.csv") \
  $(find gpurun_out/rp_${TAG}_write -name "*counter_collection.csv") gpurun_out/traffic_${TAG}.json
python tools/rocprof_agree.py gpurun_out/rp_${TAG}_bench.json $(find gpurun_out/rp_${TAG}_trace -name "*kernel_stats.csv") gpurun_out/agree_${TAG}.json
echo ROUND OK
