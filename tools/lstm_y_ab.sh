# BiLSTM line after dropping the one-layer minibatch step's f32 h writes (two runs)
set -o pipefail
for rep in 1 2; do
  timeout -k 10 300 python bench.py --model lstm --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/lstm_y_${TAG}_$rep.json 2> gpurun_out/lstm_y_${TAG}_$rep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lstm_y_${TAG}_$rep.json'));k=d['kernels_ms_per_step'];print(round(d['ms_per_step'],1), {n:round(v,1) for n,v in k.items() if 'fwdx' in n})"
done
