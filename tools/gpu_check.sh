set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo "tests exit $?" >> gpurun_out/gpu_tests.log
tail -5 gpurun_out/gpu_tests.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo BENCH FAILED; tail -30 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
