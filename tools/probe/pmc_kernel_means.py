"""Mean counter value per dispatch, per kernel, over rocprofv3 --pmc CSV directories.
Usage: python tools/probe/pmc_kernel_means.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import os
import sys


def short(name: str) -> str:
    n = name.split("(")[0]
    return n if len(n) < 70 else n[:70]


def main():
    vals = collections.defaultdict(list)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    vals[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    kernels = sorted({k for k, _ in vals})
    for k in kernels:
        print(k)
        for (kk, c), v in sorted(vals.items()):
            if kk == k:
                print(f"  {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
