"""Summarise a rocprofv3 --marker-trace CSV (roctx ranges): per range name, count / total / mean /
p50 / max duration, plus the kernel trace's total next to it when present."""
import collections
import csv
import glob
import sys


def main(d):
    rows = collections.defaultdict(list)
    for path in glob.glob(d + "/**/*marker_api_trace.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            name = r.get("Message") or r.get("Function") or r.get("Name") or "?"
            try:
                dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            except (KeyError, ValueError):
                continue
            rows[name].append(dt)
    print(f"{'range':28s} {'count':>7s} {'total_ms':>10s} {'mean_us':>9s} {'p50_us':>9s} {'max_us':>9s}")
    for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"{name[:28]:28s} {len(v):7d} {sum(v) / 1e3:10.2f} {sum(v) / len(v):9.1f} {v[len(v) // 2]:9.1f} {v[-1]:9.1f}")
    kt = collections.Counter()
    n = 0
    for path in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            kt[r["Kernel_Name"][:60]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            n += 1
    if n:
        print(f"\nkernels: {n} dispatches, {sum(kt.values()) / 1e3:.2f} ms total; top 8:")
        for k, v in kt.most_common(8):
            print(f"  {v / 1e3:9.2f} ms  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
