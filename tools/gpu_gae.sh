#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider -k gae > gpurun_out/gae_tests.log 2>&1 || { echo GAE TESTS FAILED; tail -30 gpurun_out/gae_tests.log; exit 1; }
PPO_GAE_KERNEL=reg timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider -k gae >> gpurun_out/gae_tests.log 2>&1 || { echo GAE REG TESTS FAILED; tail -30 gpurun_out/gae_tests.log; exit 1; }
grep passed gpurun_out/gae_tests.log
timeout -k 10 300 python tools/gae_sweep.py > gpurun_out/gae_sweep.jsonl 2>/dev/null || { echo SWEEP FAILED; exit 1; }
PPO_GAE_KERNEL=reg timeout -k 10 300 python tools/gae_sweep.py > gpurun_out/gae_sweep_reg.jsonl 2>/dev/null || { echo SWEEP FAILED; exit 1; }
echo lds; cat gpurun_out/gae_sweep.jsonl; echo reg; cat gpurun_out/gae_sweep_reg.jsonl
