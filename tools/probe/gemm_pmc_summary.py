"""Sum rocprofv3 counter CSVs per kernel (shortened name) over the passes in a directory."""
import collections
import csv
import glob
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
dur = collections.defaultdict(list)
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(path)):
        name = row.get("Kernel_Name", "")[:60]
        tot[name][row["Counter_Name"]] += float(row["Counter_Value"])
        cnt[name][row["Counter_Name"]] += 1
for path in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(path)):
        dur[row["Kernel_Name"][:60]].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
for name in tot:
    print(name)
    d = sorted(dur.get(name, [0]))
    print(f"   median_us {d[len(d)//2]/1e3:.1f}  n={len(d)}")
    for c, v in sorted(tot[name].items()):
        n = max(1, cnt[name][c])
        print(f"   {c:28s} per-dispatch {v / n * (1 if 'sum' in c or 'SIZE' in c else 1):,.0f}")
