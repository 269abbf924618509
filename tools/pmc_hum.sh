cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
H="--num-envs 1024 --obs-dim 376 --act-dim 17 --hidden 512,512,512 --steps 1 --warmup 1 --no-legs --no-cpu-baseline --no-timing"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_hum/p1 -o pmc --output-format csv -- python3 bench.py $H > gpurun_out/pmc_hum_p1.log 2>&1 || { tail -20 gpurun_out/pmc_hum_p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_hum/p2 -o pmc --output-format csv -- python3 bench.py $H > gpurun_out/pmc_hum_p2.log 2>&1 || { tail -20 gpurun_out/pmc_hum_p2.log; exit 1; }
for k in wide_forward_fused wide_policy_fused "wide_gemm_kernel<2, 1, 2, 4, 1"; do echo "== $k"; python3 tools/pmc_summary.py gpurun_out/pmc_hum "$k"; done
