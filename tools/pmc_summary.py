"""Average every PMC counter over the dispatches of one kernel in a tree of rocprofv3 --pmc passes.

usage: python tools/pmc_summary.py DIR KERNEL_SUBSTRING
"""
import collections
import csv
import glob
import sys


def main():
    root, needle = sys.argv[1], sys.argv[2]
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if needle in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(acc):
        v = acc[k]
        print(f"{k:32s} {sum(v) / len(v):18.1f}  (dispatches {len(v)})")


if __name__ == "__main__":
    main()
