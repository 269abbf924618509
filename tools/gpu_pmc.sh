#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over tools/micro_fused.py; summaries for the
# fused update kernel.  PASSES: space-separated comma lists.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
i=0
for P in ${PASSES:-"SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INSTS_VALU,SQ_INSTS_LDS"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc ${P//,/ } -d gpurun_out/pmc/p$i -o pmc --output-format csv -- python3 tools/micro_fused.py 10 > gpurun_out/pmc/p$i.log 2>&1 || { echo "PASS $i FAILED"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "fused_update" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(f"{k:32s} {sum(v)/len(v):16.0f}  (n={len(v)})")
PY
