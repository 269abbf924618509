#!/bin/bash
# One GPU call on the gpurun box, parameterised by STEPS (space-separated, run in order, the call
# stops at the first failing step).  Every GPU step has its own time limit.
#   tests     pytest -m gpu (K="expr" narrows it with -k)
#   smoke     __graft_entry__.smoke()
#   floor     tools/launch_floor: empty / one-load kernels and the GAE scan's bytes at its grid
#   bench     the default bench line (bf16) -> gpurun_out/bench_$TAG.json (BENCH_ARGS appended)
#   f32       bench --precision f32 -> gpurun_out/bench_${TAG}_f32.json
#   host      bench --env host (PCIe-inclusive) -> gpurun_out/bench_${TAG}_host.json
#   trace     rocprofv3 --kernel-trace --stats over the bench + timing agreement
#   traffic   FETCH_SIZE / WRITE_SIZE PMC passes over the bench -> traffic per launch
#   trafficall  the same over the bench with its config legs (every leg's roofline.traffic)
#   trafficlegs the same per workload in separate processes (LEGS="main ant hum cnn lstm"), merged
#   pmc       SQ wait / issue / LDS / MFMA counter passes over tools/micro_fused.py
#   phases    fused-update phase stamps (tools/fused_phases.py)
#   wbench    tools/wide_bench.py: the wide-path bf16 GEMMs at Humanoid shapes vs torch's matmul
#   micro     tools/micro_fused.py timing of the fused update kernel alone
#   cnn       bench.py --model cnn (pixel cheetah-run) -> bench_${TAG}_cnn.json
#   cnntrace  rocprofv3 --kernel-trace --stats over the CNN bench
#   dp2       2-rank data-parallel rehearsal on the one GPU (gloo) -> bench_${TAG}_dp2.json
#   hum       Humanoid configs[3] shard (1024 envs, O=376, A=17, 3x512) -> bench_${TAG}_hum.json
#   configs   bench lines of Ant, Humanoid 8192 on one GPU, the pixel CNN and the BiLSTM
#   humtrace  rocprofv3 --kernel-trace --stats over the Humanoid shard bench (graph replay, no events)
#   dp1       the data-parallel step sequence on one rank (PPO_DP_REHEARSE=1)
#   lstm      bench.py --model lstm (BiLSTM agent, main.py network) -> bench_${TAG}_lstm.json
#   lstmtrace rocprofv3 --kernel-trace --stats over one LSTM bench iteration
#   abmain    the headline line (no legs) per environment setting (ABSETS="A=0,B=1 ...")
#   abmodel   one model's line (MODEL) per environment setting (ABSETS="A=0,B=1 ...")
#   abhum     Humanoid shard line per value of one env knob (ABVAR, ABVALS)
#   cnnpmc    SQ counter passes over one pixel-CNN iteration (LDS-staged conv kernels)
# usage: gpurun --timeout 1200 -- 'TAG=r02 STEPS="tests bench trace traffic" bash tools/gpu.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02}
STEPS=${STEPS:-"tests smoke bench"}
fail() { echo "STEP $1 FAILED"; [ -n "$2" ] && tail -40 "$2"; exit 1; }

for S in $STEPS; do
  echo "=== $S ($(date +%T))"
  case $S in
    tests)
      timeout -k 10 1100 python -u -m pytest tests -m gpu ${NOX:--x} -v --timeout 300 --timeout-method thread \
        ${K:+-k "$K"} -s > gpurun_out/gpu_tests_${TAG}.log 2>&1 || fail tests gpurun_out/gpu_tests_${TAG}.log
      grep -E "passed|failed" gpurun_out/gpu_tests_${TAG}.log | tail -2 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
        || fail smoke gpurun_out/smoke_${TAG}.log
      tail -2 gpurun_out/smoke_${TAG}.log ;;
    floor)
      # the launch / memory floor under the GAE scan (tools/launch_floor.hip): events and rocprofv3
      timeout -k 10 120 ./tools/launch_floor 400 > gpurun_out/floor_${TAG}.json 2> gpurun_out/floor_${TAG}.err \
        || fail floor gpurun_out/floor_${TAG}.err
      cat gpurun_out/floor_${TAG}.json
      timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_${TAG}_floor -o floor --output-format csv \
        -- ./tools/launch_floor 400 > gpurun_out/rp_${TAG}_floor.log 2>&1 || fail floortrace gpurun_out/rp_${TAG}_floor.log
      cat $(find gpurun_out/rp_${TAG}_floor -name "*kernel_stats.csv") ;;
    bench)
      timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
        || fail bench gpurun_out/bench_${TAG}.err
      cat gpurun_out/bench_${TAG}.json ;;
    f32)
      timeout -k 10 400 python bench.py --precision f32 --no-cpu-baseline > gpurun_out/bench_${TAG}_f32.json \
        2> gpurun_out/bench_${TAG}_f32.err || fail f32 gpurun_out/bench_${TAG}_f32.err
      cat gpurun_out/bench_${TAG}_f32.json ;;
    host)
      timeout -k 10 400 python bench.py --env host --no-cpu-baseline > gpurun_out/bench_${TAG}_host.json \
        2> gpurun_out/bench_${TAG}_host.err || fail host gpurun_out/bench_${TAG}_host.err
      cat gpurun_out/bench_${TAG}_host.json ;;
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_${TAG}_trace -o bench --output-format csv \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/rp_${TAG}_bench.json \
        2> gpurun_out/rp_${TAG}_trace.log || fail trace gpurun_out/rp_${TAG}_trace.log
      python tools/rocprof_agree.py gpurun_out/rp_${TAG}_bench.json \
        $(find gpurun_out/rp_${TAG}_trace -name "*kernel_stats.csv") gpurun_out/agree_${TAG}.json ;;
    traffic)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/rp_${TAG}_fetch -o fetch --output-format csv \
        -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-timing --no-legs \
        > gpurun_out/rp_${TAG}_fetch.log 2>&1 || fail fetch gpurun_out/rp_${TAG}_fetch.log
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/rp_${TAG}_write -o write --output-format csv \
        -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-timing --no-legs \
        > gpurun_out/rp_${TAG}_write.log 2>&1 || fail write gpurun_out/rp_${TAG}_write.log
      python tools/pmc_traffic.py $(find gpurun_out/rp_${TAG}_fetch -name "*counter_collection.csv") \
        $(find gpurun_out/rp_${TAG}_write -name "*counter_collection.csv") gpurun_out/traffic_${TAG}.json ;;
    trafficall)
      # FETCH_SIZE / WRITE_SIZE passes over the bench INCLUDING its config legs (Ant, Humanoid
      # shard, pixel CNN, BiLSTM): per-kernel traffic for every leg's roofline -> bench_traffic.json
      timeout -s KILL 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/rp_${TAG}_fetchall -o fetch --output-format csv \
        -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --leg-steps 1 \
        > gpurun_out/rp_${TAG}_fetchall.log 2>&1 || fail fetchall gpurun_out/rp_${TAG}_fetchall.log
      timeout -s KILL 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/rp_${TAG}_writeall -o write --output-format csv \
        -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --leg-steps 1 \
        > gpurun_out/rp_${TAG}_writeall.log 2>&1 || fail writeall gpurun_out/rp_${TAG}_writeall.log
      python tools/pmc_traffic.py $(find gpurun_out/rp_${TAG}_fetchall -name "*counter_collection.csv") \
        $(find gpurun_out/rp_${TAG}_writeall -name "*counter_collection.csv") gpurun_out/trafficall_${TAG}.json ;;
    trafficlegs)
      # FETCH_SIZE / WRITE_SIZE passes per workload (LEGS="main ant hum cnn lstm"), one process each,
      # merged into gpurun_out/trafficlegs_${TAG}.json (copy it to bench_traffic.json)
      BASE="--steps 1 --warmup 1 --no-cpu-baseline --no-timing --no-legs --no-graphs"  # rocprofv3 --pmc crashed in hipGraph replay
      outs=""
      for L in ${LEGS:-main ant hum lstm cnn}; do
        case $L in
          main) A="" ;;
          ant) A="--num-envs 4096 --obs-dim 27 --act-dim 8" ;;
          hum) A="--num-envs 1024 --obs-dim 376 --act-dim 17 --hidden 512,512,512 --batch 8192" ;;
          cnn) A="--model cnn" ;;
          lstm) A="--model lstm ${LSTM_TRAFFIC_ARGS}" ;;  # e.g. --epochs 1: same per-launch shapes, fewer dispatches
        esac
        for C in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
          # the profiled run writes only to its log: a heartbeat on stdout keeps the call alive
          timeout -s KILL 600 rocprofv3 --pmc $C -d gpurun_out/rp_${TAG}_${L}_$C -o pmc --output-format csv \
            -- python3 bench.py $BASE $A > gpurun_out/rp_${TAG}_${L}_$C.log 2>&1 &
          pid=$!
          while kill -0 $pid 2>/dev/null; do sleep 20; echo "  $L $C running ($(date +%T))"; done
          wait $pid || fail "traffic $L $C" gpurun_out/rp_${TAG}_${L}_$C.log
        done
        if [ -z "$COUNTERS" ]; then
          python tools/pmc_traffic.py $(find gpurun_out/rp_${TAG}_${L}_FETCH_SIZE -name "*counter_collection.csv") \
            $(find gpurun_out/rp_${TAG}_${L}_WRITE_SIZE -name "*counter_collection.csv") gpurun_out/traffic_${TAG}_$L.json \
            > /dev/null
          outs="$outs $( [ $L = hum ] && echo humanoid || echo $L )=gpurun_out/traffic_${TAG}_$L.json"
        fi
      done
      [ -n "$outs" ] && python tools/merge_traffic.py gpurun_out/trafficlegs_${TAG}.json $outs ;;
    pmc)
      i=0
      # one pass per space-separated word (at most 8 SQ_ counters each)
      PASSES=${PASSES:-"SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INSTS_VALU,SQ_INSTS_LDS SQ_INSTS_MFMA,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE"}
      for P in $PASSES; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc ${P//,/ } -d gpurun_out/pmc_${TAG}/p$i -o pmc --output-format csv \
          -- python3 tools/micro_fused.py 10 > gpurun_out/pmc_${TAG}_p$i.log 2>&1 || fail pmc$i gpurun_out/pmc_${TAG}_p$i.log
      done
      python3 tools/pmc_summary.py gpurun_out/pmc_${TAG} fused_update > gpurun_out/pmc_${TAG}.txt
      cat gpurun_out/pmc_${TAG}.txt ;;
    cnnpmc)
      # SQ counter passes over one pixel-CNN iteration (the LDS-staged conv kernels)
      i=0
      PASSES=${PASSES:-"SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INSTS_VALU,SQ_INSTS_LDS SQ_INSTS_MFMA,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_BUSY_CYCLES,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,GRBM_GUI_ACTIVE"}
      for P in $PASSES; do
        i=$((i+1))
        timeout -s KILL 300 rocprofv3 --pmc ${P//,/ } -d gpurun_out/cpmc_${TAG}/p$i -o pmc --output-format csv \
          -- python3 bench.py --model cnn --steps 1 --warmup 1 --no-cpu-baseline --no-timing --no-legs \
          > gpurun_out/cpmc_${TAG}_p$i.log 2>&1 || fail cnnpmc$i gpurun_out/cpmc_${TAG}_p$i.log
      done
      for KN in fwd_lds_kernel dgrad_lds_kernel wgrad_lds_kernel pixel_fwd pixel_wgrad; do
        echo "--- $KN"; python3 tools/pmc_summary.py gpurun_out/cpmc_${TAG} $KN
      done > gpurun_out/cpmc_${TAG}.txt
      cat gpurun_out/cpmc_${TAG}.txt ;;
    phases)
      timeout -k 10 200 python tools/fused_phases.py > gpurun_out/phases_${TAG}.txt 2>&1 || fail phases gpurun_out/phases_${TAG}.txt
      cat gpurun_out/phases_${TAG}.txt ;;
    lstm)
      timeout -k 10 600 python bench.py --model lstm $LSTM_ARGS > gpurun_out/bench_${TAG}_lstm.json \
        2> gpurun_out/bench_${TAG}_lstm.err || fail lstm gpurun_out/bench_${TAG}_lstm.err
      cat gpurun_out/bench_${TAG}_lstm.json ;;
    lstmtrace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_${TAG}_lstm -o lstm --output-format csv \
        -- python3 bench.py --model lstm --steps 1 --warmup 1 $LSTM_ARGS > gpurun_out/rp_${TAG}_lstm.json \
        2> gpurun_out/rp_${TAG}_lstm.log || fail lstmtrace gpurun_out/rp_${TAG}_lstm.log
      head -12 $(find gpurun_out/rp_${TAG}_lstm -name "*kernel_stats.csv") ;;
    abhum)
      # A/B of one environment knob on the Humanoid shard line: ABVAR=NAME ABVALS="v1 v2 ..."
      for V in $ABVALS; do
        env $ABVAR=$V timeout -k 10 500 python bench.py --num-envs 1024 --obs-dim 376 --act-dim 17 \
          --hidden 512,512,512 --batch ${HUM_BATCH:-8192} --steps 3 --warmup 2 --no-legs --no-cpu-baseline \
          > gpurun_out/bench_${TAG}_hum_$V.json 2> gpurun_out/bench_${TAG}_hum_$V.err \
          || fail abhum gpurun_out/bench_${TAG}_hum_$V.err
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'])" \
          gpurun_out/bench_${TAG}_hum_$V.json
      done ;;
    abmain)
      # A/B of environment settings on the headline line (no legs): ABSETS="X=0,Y=1 X=1,Y=1 ..."
      i=0
      for SET in $ABSETS; do
        i=$((i+1))
        env ${SET//,/ } timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline $BENCH_ARGS \
          > gpurun_out/bench_${TAG}_m$i.json 2> gpurun_out/bench_${TAG}_m$i.err \
          || fail "abmain $SET" gpurun_out/bench_${TAG}_m$i.err
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernels_ms_per_step',{}); print(sys.argv[2], d['value'], d['ms_per_step'], {n: round(v, 4) for n, v in k.items() if v > 0.1})" \
          gpurun_out/bench_${TAG}_m$i.json "$SET"
      done ;;
    abmodel)
      # A/B of environment settings on one model's line: MODEL=lstm|cnn ABSETS="X=0,Y=1 X=1,Y=1 ..."
      i=0
      for SET in $ABSETS; do
        i=$((i+1))
        env ${SET//,/ } timeout -k 10 500 python bench.py --model ${MODEL:-lstm} --steps 3 --warmup 2 \
          --no-cpu-baseline > gpurun_out/bench_${TAG}_ab$i.json 2> gpurun_out/bench_${TAG}_ab$i.err \
          || fail "abmodel $SET" gpurun_out/bench_${TAG}_ab$i.err
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
          gpurun_out/bench_${TAG}_ab$i.json "$SET"
      done ;;
    cnn)
      timeout -k 10 600 python bench.py --model cnn $CNN_ARGS > gpurun_out/bench_${TAG}_cnn.json \
        2> gpurun_out/bench_${TAG}_cnn.err || fail cnn gpurun_out/bench_${TAG}_cnn.err
      cat gpurun_out/bench_${TAG}_cnn.json ;;
    cnntrace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_${TAG}_cnn -o cnn --output-format csv \
        -- python3 bench.py --model cnn --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rp_${TAG}_cnn.json \
        2> gpurun_out/rp_${TAG}_cnn.log || fail cnntrace gpurun_out/rp_${TAG}_cnn.log
      head -16 $(find gpurun_out/rp_${TAG}_cnn -name "*kernel_stats.csv") ;;
    dp2)
      PPO_BENCH_BACKEND=gloo PPO_BENCH_ONE_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
        --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_dp2.json \
        2> gpurun_out/bench_${TAG}_dp2.err || fail dp2 gpurun_out/bench_${TAG}_dp2.err
      cat gpurun_out/bench_${TAG}_dp2.json ;;
    dp1)
      PPO_DP_REHEARSE=1 timeout -k 10 400 python bench.py --no-cpu-baseline --no-legs > gpurun_out/bench_${TAG}_dp1.json \
        2> gpurun_out/bench_${TAG}_dp1.err || fail dp1 gpurun_out/bench_${TAG}_dp1.err
      cat gpurun_out/bench_${TAG}_dp1.json ;;
    hum)
      timeout -k 10 500 python bench.py --num-envs 1024 --obs-dim 376 --act-dim 17 --hidden 512,512,512 \
        --batch ${HUM_BATCH:-8192} --steps 3 --warmup 2 --no-legs --no-cpu-baseline > gpurun_out/bench_${TAG}_hum.json \
        2> gpurun_out/bench_${TAG}_hum.err || fail hum gpurun_out/bench_${TAG}_hum.err
      cat gpurun_out/bench_${TAG}_hum.json ;;
    humtrace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_${TAG}_hum -o hum --output-format csv \
        -- python3 bench.py --num-envs 1024 --obs-dim 376 --act-dim 17 --hidden 512,512,512 \
        --steps 2 --warmup 1 --no-legs --no-cpu-baseline --no-timing > gpurun_out/rp_${TAG}_hum.json \
        2> gpurun_out/rp_${TAG}_hum.log || fail humtrace gpurun_out/rp_${TAG}_hum.log
      head -25 $(find gpurun_out/rp_${TAG}_hum -name "*kernel_stats.csv") | cut -c1-160 ;;
    configs)
      # the BASELINE configs beside the headline (profiles/r03_configs.md): Ant, Humanoid 8192 on
      # one GPU, the pixel CNN, the main.py BiLSTM
      timeout -k 10 300 python bench.py --obs-dim 27 --act-dim 8 --no-legs --no-cpu-baseline \
        > gpurun_out/bench_${TAG}_ant.json 2> gpurun_out/bench_${TAG}_ant.err || fail ant gpurun_out/bench_${TAG}_ant.err
      timeout -k 10 400 python bench.py --num-envs 8192 --obs-dim 376 --act-dim 17 --hidden 512,512,512 \
        --steps 2 --warmup 1 --no-legs --no-cpu-baseline > gpurun_out/bench_${TAG}_hum8k.json \
        2> gpurun_out/bench_${TAG}_hum8k.err || fail hum8k gpurun_out/bench_${TAG}_hum8k.err
      timeout -k 10 500 python bench.py --model cnn --steps 2 --warmup 1 --no-cpu-baseline \
        > gpurun_out/bench_${TAG}_cnn.json 2> gpurun_out/bench_${TAG}_cnn.err || fail cnn gpurun_out/bench_${TAG}_cnn.err
      timeout -k 10 500 python bench.py --model lstm --steps 2 --warmup 1 \
        > gpurun_out/bench_${TAG}_lstm.json 2> gpurun_out/bench_${TAG}_lstm.err || fail lstm gpurun_out/bench_${TAG}_lstm.err
      for c in ant hum8k cnn lstm; do cut -c1-200 gpurun_out/bench_${TAG}_$c.json; done ;;
    wbench)
      timeout -k 10 200 python tools/wide_bench.py 20 > gpurun_out/wbench_${TAG}.txt 2>&1 || fail wbench gpurun_out/wbench_${TAG}.txt
      cat gpurun_out/wbench_${TAG}.txt ;;
    micro)
      timeout -k 10 200 python tools/micro_fused.py 20 > gpurun_out/micro_${TAG}.txt 2>&1 || fail micro gpurun_out/micro_${TAG}.txt
      cat gpurun_out/micro_${TAG}.txt ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "ALL STEPS OK"
