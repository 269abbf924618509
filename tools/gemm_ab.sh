#!/bin/bash
# A/B the large-tile GEMM variants in one box session (same device), printing per-class ms/iter.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in "2 0" "1 0" "2 1" "1 1" "2 0"; do
  set -- $cfg
  PPO_GEMM_NBUF=$1 PPO_GEMM_WIDE=$2 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$1_$2.json 2> gpurun_out/ab_err.log || { echo "FAILED nbuf=$1 wide=$2"; tail -5 gpurun_out/ab_err.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$1_$2.json')); c=d['kernel_classes_ms_per_step']; print('nbuf=$1 wide=$2', round(d['ms_per_step'],1), {k: round(v,1) for k,v in c.items()})"
done
