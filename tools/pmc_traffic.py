"""HBM traffic per launch from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, one pass each --
they do not fit one pass on gfx950) over the bench command.

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are KB at the L2's memory side;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so
    traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   bytes per dispatch.
Infinity-Cache hits are counted as traffic by these counters.

usage: python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv OUT.json
"""
import csv
import json
import sys
from collections import defaultdict


def kernel_key(name: str) -> str:
    """'void ppo::gemm_f32_kernel<2, 2, ...>(ppo::GemmBatch)' -> 'gemm_f32_kernel<2, 2, ...>'."""
    if name.startswith("void "):
        name = name[5:]
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            name = name[:i]
            break
    # drop every namespace qualifier outside the template arguments (ppo::, ppo::lstm::, ...)
    depth, cut = 0, 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif depth == 0 and name.startswith("::", i):
            cut = i + 2
    return name[cut:]


_LAYER = {"32, 20,": "L2", "64, 9,": "L3"}


def bench_key(key: str) -> str:
    """The name bench.py's event records use: namespaces dropped ('conv::pixel_wgrad_kernel' ->
    'pixel_wgrad_kernel'), and the LDS-staged conv kernels named by layer
    ('conv::dgrad_lds_kernel<ppo::conv::DgGeo<32, 20, ...>>' -> 'dgrad_lds_kernel<L2>')."""
    head, sep, rest = key.partition("<")
    if head.split("::")[0] in ("conv", "lstm", "f4", "cnn", "wide", "fu"):  # the engine's namespaces
        head = head.split("::")[-1]
    if head in ("fwd_lds_kernel", "dgrad_lds_kernel", "wgrad_lds_kernel", "dg_pack_kernel",
                "fw_pack_kernel"):
        for sig, layer in _LAYER.items():
            if sig in rest:
                return f"{head}<{layer}>" if "lds" in head else head
    return head + sep + rest


def per_kernel(path: str, counter: str) -> dict:
    tot, cnt = defaultdict(float), defaultdict(int)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            k = bench_key(kernel_key(row["Kernel_Name"]))
            tot[k] += float(row["Counter_Value"])
            cnt[k] += 1
    return {k: (tot[k] / cnt[k], cnt[k]) for k in tot}


def main():
    fetch_csv, write_csv, out = sys.argv[1:4]
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    res = {"formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 B per dispatch (gfx950 FETCH_SIZE "
                      "counts half of a wide coalesced read; MI355X_MICROARCH.md HBM section)",
           "sources": [fetch_csv, write_csv], "bytes_per_launch": {}, "fetch_kb": {},
           "write_kb": {}, "dispatches": {}}
    for k in sorted(set(fetch) & set(write)):
        f, nf = fetch[k]
        w, nw = write[k]
        res["bytes_per_launch"][k] = (2.0 * f + w) * 1024.0
        res["fetch_kb"][k] = f
        res["write_kb"][k] = w
        res["dispatches"][k] = min(nf, nw)
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1, sort_keys=True)
    for k, v in sorted(res["bytes_per_launch"].items(), key=lambda kv: -kv[1])[:15]:
        print(f"{v / 1e6:12.3f} MB  {k}")


if __name__ == "__main__":
    main()
