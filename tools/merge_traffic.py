"""Merge per-workload PMC traffic tables (tools/pmc_traffic.py outputs) into the one table bench.py
reads (bench_traffic.json): the headline's kernels at the top level (`bytes_per_launch`), every
config leg's under `by_workload[leg]` -- the layered GEMM instantiations are shared by the pixel
and BiLSTM heads with different shapes, so a leg's roofline only reads its own workload's bytes.

usage: python tools/merge_traffic.py OUT.json main=MAIN.json [ant=ANT.json humanoid=... cnn=... lstm=...]
"""
import json
import sys


def main():
    out = sys.argv[1]
    res = {"formula": None, "sources": {}, "bytes_per_launch": {}, "by_workload": {},
           "dispatches": {}}
    for arg in sys.argv[2:]:
        name, path = arg.split("=", 1)
        with open(path) as f:
            t = json.load(f)
        res["formula"] = t.get("formula", res["formula"])
        res["sources"][name] = path
        table = t.get("bytes_per_launch", {})
        if name == "main":
            res["bytes_per_launch"] = table
            res["dispatches"] = t.get("dispatches", {})
        else:
            res["by_workload"][name] = table
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(f"{out}: headline {len(res['bytes_per_launch'])} kernels, legs {sorted(res['by_workload'])}")


if __name__ == "__main__":
    main()
