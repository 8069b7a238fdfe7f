"""Per-decode-step kernel summary of a rocprofv3 kernel trace of tools/bench_models.py llama (the last
31 steps, cut at each step's embedding launch).  Usage: decode_step_summary.py <trace.csv> [title]"""
import collections
import csv
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:90]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    idx = [i for i, (_, _, n) in enumerate(rows) if "embedding" in n]
    seg = rows[idx[-31]:]
    steps = 31
    span = (seg[-1][1] - seg[0][0]) / 1e3 / steps
    agg = collections.defaultdict(lambda: [0, 0.0])
    for s, e, n in seg:
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values()) / steps
    if len(sys.argv) > 2:
        print(sys.argv[2])
    print(f"span per step {span:.1f} us, kernel sum {tot:.1f} us, {len(seg) / steps:.0f} kernels per step")
    for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
        print(f"{t / steps:9.1f} us  n={c / steps:5.1f}  avg={t / c:7.2f}  {n}")


if __name__ == "__main__":
    main()
