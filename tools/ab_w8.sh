#!/bin/bash
# A/B of the layered GEMMs' 128x128 tile: 4 waves (default) vs 8 waves (PPO_GEMM_W8=1) on the
# LSTM line, the f32 leg and the CNN line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 0 1; do
  PPO_GEMM_W8=$w timeout -k 10 300 python bench.py --model lstm --steps 2 --warmup 1 > gpurun_out/ab_w8_${w}_lstm.json 2> gpurun_out/ab_w8_${w}_lstm.err || { tail -5 gpurun_out/ab_w8_${w}_lstm.err; exit 1; }
  PPO_GEMM_W8=$w timeout -k 10 300 python bench.py --precision f32 --steps 3 --warmup 1 --no-legs --no-cpu-baseline > gpurun_out/ab_w8_${w}_f32.json 2> gpurun_out/ab_w8_${w}_f32.err || { tail -5 gpurun_out/ab_w8_${w}_f32.err; exit 1; }
  PPO_GEMM_W8=$w timeout -k 10 300 python bench.py --model cnn --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_w8_${w}_cnn.json 2> gpurun_out/ab_w8_${w}_cnn.err || { tail -5 gpurun_out/ab_w8_${w}_cnn.err; exit 1; }
done
for f in gpurun_out/ab_w8_*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(round(d['value']), round(d['ms_per_step'],2))")"; done
