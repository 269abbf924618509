set -o pipefail
for c in 0 1 3 10 12; do
  if [ $c = 0 ]; then unset PPO_WIDE_CFG; else export PPO_WIDE_CFG=$c; fi
  timeout -k 10 300 python bench.py --model lstm --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lstm_cfg_r06t_$c.json 2> gpurun_out/lstm_cfg_r06t_$c.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lstm_cfg_r06t_$c.json'));k=d['kernels_ms_per_step'];print($c, round(d['ms_per_step'],1), {n:round(v,1) for n,v in k.items() if 'wide' in n})"
done
