# A/B of the BiLSTM weight-gradient split count (PPO_LSTM_SPLITS), alternating, one process each
set -o pipefail
for rep in 1 2; do
for c in 32 16; do
  PPO_LSTM_SPLITS=$c timeout -k 10 300 python bench.py --model lstm --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/lstm_splits_${TAG}_${c}_$rep.json 2> gpurun_out/lstm_splits_${TAG}_${c}_$rep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lstm_splits_${TAG}_${c}_$rep.json'));k=d['kernels_ms_per_step'];print($c, round(d['ms_per_step'],1), {n:round(v,1) for n,v in k.items() if 'reduce' in n or 'wide_gemm' in n or 'gemm_bf16_kernel<2, 1, 2, 4, 64, 1' in n})"
done
done
