#!/bin/bash
# Kernel trace + PMC passes over tools/profile_minibatch.py; summaries land in gpurun_out/prof*.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o trace --output-format csv \
  -- python3 tools/profile_minibatch.py --mode iter --reps 2 > gpurun_out/prof_trace.log 2>&1 || { echo TRACE FAILED; tail -20 gpurun_out/prof_trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d gpurun_out/prof_pmc1 -o pmc1 --output-format csv -- python3 tools/profile_minibatch.py --mode mb --reps 1 > gpurun_out/prof_pmc1.log 2>&1 || { echo PMC1 FAILED; tail -20 gpurun_out/prof_pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d gpurun_out/prof_pmc2 -o pmc2 --output-format csv -- python3 tools/profile_minibatch.py --mode mb --reps 1 > gpurun_out/prof_pmc2.log 2>&1 || { echo PMC2 FAILED; tail -20 gpurun_out/prof_pmc2.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE \
  -d gpurun_out/prof_pmc3 -o pmc3 --output-format csv -- python3 tools/profile_minibatch.py --mode mb --reps 1 > gpurun_out/prof_pmc3.log 2>&1 || { echo PMC3 FAILED; tail -20 gpurun_out/prof_pmc3.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE \
  -d gpurun_out/prof_pmc4 -o pmc4 --output-format csv -- python3 tools/profile_minibatch.py --mode mb --reps 1 > gpurun_out/prof_pmc4.log 2>&1 || { echo PMC4 FAILED; tail -20 gpurun_out/prof_pmc4.log; exit 1; }
find gpurun_out/prof_* -name "*.csv" | head -20
echo PROFILE OK
