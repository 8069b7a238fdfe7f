"""Whole-forward PMC totals from rocprofv3 counter CSVs of tools/probe/forward_probe.py: per
counter, the sum over the kernels of ONE forward (total / forwards), plus kernel time."""
import collections
import csv
import glob
import sys


def main():
    root, forwards = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3
    tot = collections.defaultdict(float)
    seen = set()
    dur = 0.0
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            if key not in seen:
                seen.add(key)
                dur += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    out = {k: v / forwards for k, v in sorted(tot.items())}
    out["kernel_us_per_forward"] = dur / forwards
    out["dispatches_per_forward"] = len(seen) / forwards
    for k, v in out.items():
        print(f"{k:32s} {v:,.1f}")


if __name__ == "__main__":
    main()
