#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for eb in 16 8 4 32; do
  PPO_GAE_EB=$eb timeout -k 10 120 python tools/gae_sweep.py 2>/dev/null | head -2 | sed "s/^/eb=$eb /" || true
done
timeout -k 10 120 python tools/gae_sweep.py 2>/dev/null > gpurun_out/gae_sweep_final.jsonl; cat gpurun_out/gae_sweep_final.jsonl
