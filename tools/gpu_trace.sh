#!/bin/bash
# rocprofv3 kernel-trace stats over a short bench run (all kernels incl. graph-replayed rollout).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-tr}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_${TAG} -o bench --output-format csv \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rp_${TAG}_bench.json 2> gpurun_out/rp_${TAG}.log || { echo TRACE FAILED; tail -20 gpurun_out/rp_${TAG}.log; exit 1; }
python - <<PY
import csv, glob
f = glob.glob("gpurun_out/rp_${TAG}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms per iteration (4 iterations):", tot / 4e6)
for r in rows[:16]:
    print(f"{float(r['TotalDurationNs'])/4e6:9.3f} ms/it {int(r['Calls'])//4:>6}/it {float(r['AverageNs'])/1e3:9.2f} us  {r['Name'][:100]}")
PY
