# A/B of the BiLSTM rollout's paired step launches (PPO_LSTM_PAIR_STEPS 0 / 1), alternating
set -o pipefail
for rep in 1 2; do
for c in 0 1; do
  PPO_LSTM_PAIR_STEPS=$c timeout -k 10 300 python bench.py --model lstm --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/lstm_pair_${TAG}_${c}_$rep.json 2> gpurun_out/lstm_pair_${TAG}_${c}_$rep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lstm_pair_${TAG}_${c}_$rep.json'));k=d['kernels_ms_per_step'];print($c, round(d['ms_per_step'],1), {n:round(v,1) for n,v in k.items() if 'rollout' in n})"
done
done
