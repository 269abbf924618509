# A/B of the Humanoid shard's layer-0 WGRAD split count (PPO_WIDE_SPLITS0 8 / 16)
set -o pipefail
A="--num-envs 1024 --obs-dim 376 --act-dim 17 --hidden 512,512,512 --batch 8192 --steps 3 --warmup 1 --no-cpu-baseline --no-legs"
for rep in 1 2; do
for c in 8 16; do
  PPO_WIDE_SPLITS0=$c timeout -k 10 300 python bench.py $A > gpurun_out/hum_s0_${TAG}_${c}_$rep.json 2> gpurun_out/hum_s0_${TAG}_${c}_$rep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/hum_s0_${TAG}_${c}_$rep.json'));k=d['kernels_ms_per_step'];print($c, round(d['ms_per_step'],2), {n:round(v,2) for n,v in k.items() if 'gemm' in n or 'reduce' in n})"
done
done
