#!/bin/bash
# Fused-kernel tests (incl. determinism), policy timing probe, phase stamps, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bf16 or staged or graphs or fused or deterministic or observe" > gpurun_out/check2.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/check2.log; exit 1; }
tail -1 gpurun_out/check2.log
timeout -k 10 200 python tools/micro_policy.py 2>&1 | grep "N=  4096" || { echo POLICY FAILED; exit 1; }
tools/gpu_perf.sh
