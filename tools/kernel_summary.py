"""Aggregate a rocprofv3 ``--kernel-trace`` CSV (or its SQLite ``results.db``) by kernel name: total/avg µs and call count,
optionally restricted to the last ``--window`` kernels and normalised per ``--per`` steps.
Usage: python tools/kernel_summary.py <dir-or-csv> [--window N] [--per K] [--top 30]"""
import argparse
import collections
import csv
import glob
import os


def load_db(path):
    """rocprofv3's default SQLite output (``*_results.db``): the ``kernels`` view."""
    import sqlite3

    con = sqlite3.connect(path)
    try:
        return sorted((int(s), int(e), n) for s, e, n in con.execute("select start, end, name from kernels"))
    finally:
        con.close()


def load(path):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*results.db"), recursive=True)
        cands = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if dbs and not cands:
            return load_db(dbs[0])
        if not cands:
            raise SystemExit(f"no kernel_trace.csv / results.db under {path}")
        path = cands[0]
    if path.endswith(".db"):
        return load_db(path)
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    depth, out = 0, []
    for ch in name:  # cut at the argument list, keeping template arguments
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    return "".join(out)[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--window", type=int, default=0, help="only the last N kernels")
    ap.add_argument("--per", type=float, default=1.0, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--last-of", default="", help="start at the --per-th last launch of a kernel whose name "
                                                   "contains this (e.g. the first kernel of a forward)")
    a = ap.parse_args()
    rows = load(a.path)
    if a.window:
        rows = rows[-a.window:]
    if a.last_of:
        starts = [i for i, (_s, _e, n) in enumerate(rows) if a.last_of in n]
        if len(starts) < int(a.per):
            raise SystemExit(f"only {len(starts)} launches of {a.last_of!r}")
        rows = rows[starts[-int(a.per)]:]
    agg = collections.defaultdict(lambda: [0.0, 0])
    for s, e, n in rows:
        agg[short(n)][0] += (e - s) / 1e3
        agg[short(n)][1] += 1
    tot = sum(v[0] for v in agg.values())
    span = (rows[-1][1] - rows[0][0]) / 1e3 if rows else 0.0
    busy, cur_s, cur_e = 0.0, None, None  # union of kernel intervals: time the GPU ran >= 1 kernel
    for s, e, _n in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    print(f"kernels {len(rows)}  kernel-sum {tot / a.per:.1f} us  span {span / a.per:.1f} us  "
          f"busy {busy / 1e3 / a.per:.1f} us  (per {a.per:g})")
    for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{t / a.per:10.1f} us  n={c / a.per:7.1f}  avg={t / c:8.2f} us  {n}")


if __name__ == "__main__":
    main()
