"""Merge per-workload PMC traffic tables (tools/pmc_traffic.py outputs) into the one table bench.py
reads (bench_traffic.json).  Later inputs override earlier ones for a kernel name both contain:
list the headline first and the legs after it, so each leg's dominant kernel carries the bytes of
the leg's own shapes (the layered GEMM instantiations are shared by the pixel and BiLSTM heads).

usage: python tools/merge_traffic.py OUT.json IN1.json [IN2.json ...]
"""
import json
import sys


def main():
    out, ins = sys.argv[1], sys.argv[2:]
    res = {"formula": None, "sources": [], "bytes_per_launch": {}, "fetch_kb": {}, "write_kb": {},
           "dispatches": {}, "workload_of": {}}
    for path in ins:
        with open(path) as f:
            t = json.load(f)
        res["formula"] = t.get("formula", res["formula"])
        res["sources"].append(path)
        for key in ("bytes_per_launch", "fetch_kb", "write_kb", "dispatches"):
            res[key].update(t.get(key, {}))
        for k in t.get("bytes_per_launch", {}):
            res["workload_of"][k] = path
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(f"{out}: {len(res['bytes_per_launch'])} kernels from {len(ins)} tables")


if __name__ == "__main__":
    main()
