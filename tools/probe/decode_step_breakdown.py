"""Per-kernel breakdown of the LAST decode step in a rocprofv3 kernel trace (a step starts at the
embedding kernel): calls, total and mean microseconds per kernel name."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "embed" in r["Kernel_Name"].lower()]
step = rows[starts[-1]:]


def name(k):
    return re.split(r"\(", k.replace("void ", "").replace("(anonymous namespace)::", ""))[0][:80]


agg = collections.OrderedDict()
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg.setdefault(name(r["Kernel_Name"]), [0, 0.0])
    a[0] += 1
    a[1] += d
wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{c:4d} {d:9.1f} {d / c:7.2f}  {n}")
print(f"kernels {len(step)}  wall_us {wall:.1f}")
