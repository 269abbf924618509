"""Cross-check bench.py's live per-kernel event timing against a rocprofv3 --kernel-trace --stats
summary of the same command: for the roofline kernel and the GAE kernel, print the bench's mean
launch duration next to rocprof's AverageNs for the same kernel name.

usage: python tools/rocprof_agree.py BENCH.json KERNEL_STATS.csv [OUT.json]
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import kernel_key  # noqa: E402


def main():
    bench_path, stats_path = sys.argv[1:3]
    with open(bench_path) as f:
        line = json.loads([ln for ln in f if ln.startswith("{")][-1])
    stats = {}
    with open(stats_path) as f:
        for row in csv.DictReader(f):
            stats[kernel_key(row["Name"])] = row
    out = {"bench": bench_path, "rocprof": stats_path, "kernels": {}}
    for key in ("roofline", "gae_roofline"):
        r = line.get(key)
        if not r:
            continue
        s = stats.get(r["kernel"])
        rec = {"bench_avg_us": r["avg_launch_us"], "bench_launches": r["launches"]}
        if s:
            rec["rocprof_avg_us"] = float(s["AverageNs"]) / 1e3
            rec["rocprof_calls"] = int(s["Calls"])
            rec["ratio_bench_over_rocprof"] = rec["bench_avg_us"] / rec["rocprof_avg_us"]
        out["kernels"][r["kernel"]] = rec
        print(key, r["kernel"], json.dumps(rec))
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
