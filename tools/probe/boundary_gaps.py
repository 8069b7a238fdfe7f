"""What kernel boundaries cost a ResNet-50 forward, from a rocprofv3 ``--kernel-trace`` CSV of the bench.

Per stream (= per engine slot), the dispatches are cut into forwards at each ``stem_pool`` kernel; for
every forward this sums the kernel durations and the idle gaps between one kernel's end and the next
kernel's start on the same stream (the launch boundary as the batch sees it), over the whole forward
and over its layer-4 tail (the kernels after the last layer-3 one: position >= --l4-from).  This is
the upper bound of what fusing launches (one persistent / stream-K launch per bottleneck) can remove
from a batch's latency: a fused launch keeps each stage's tiles and K loops, it only removes the
boundaries.  Usage: python tools/probe/boundary_gaps.py <kernel_trace.csv> [--l4-from N] [--skip F]"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--l4-from", type=int, default=0,
                    help="forward kernel index where layer 4 starts (0: from the kernel names, see below)")
    ap.add_argument("--skip", type=int, default=10, help="forwards per stream to skip (warm-up)")
    a = ap.parse_args()
    by_stream = collections.defaultdict(list)
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            by_stream[int(r["Stream_Id"])].append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    fwds = []
    for sid, rows in by_stream.items():
        rows.sort()
        cur = None
        for s, e, n in rows:
            if "stem_pool" in n:
                if cur:
                    fwds.append((sid, cur))
                cur = []
            if cur is not None and "h2d_pull" not in n and "d2h_push" not in n:
                cur.append((s, e, n))
        if cur:
            fwds.append((sid, cur))
    # full forwards only (stem ... head_finish), warm-up forwards dropped per stream
    seen = collections.Counter()
    keep = []
    for sid, ks in fwds:
        if not ks or "head_finish" not in ks[-1][2]:
            continue
        seen[sid] += 1
        if seen[sid] > a.skip:
            keep.append(ks)
    if not keep:
        print("no complete forwards")
        return
    nk = collections.Counter(len(k) for k in keep).most_common(1)[0][0]
    keep = [k for k in keep if len(k) == nk]
    l4 = a.l4_from or nk - 10  # ResNet-50 here: layer 4 = the last 8 conv launches + the 2 head launches
    rows = []
    for ks in keep:
        dur = sum(e - s for s, e, _ in ks) / 1e3
        gaps = [max(0, ks[i + 1][0] - ks[i][1]) / 1e3 for i in range(len(ks) - 1)]
        span = (ks[-1][1] - ks[0][0]) / 1e3
        dur4 = sum(e - s for s, e, _ in ks[l4:]) / 1e3
        gap4 = sum(gaps[l4 - 1:])
        rows.append((span, dur, sum(gaps), max(gaps), dur4, gap4, statistics.median(gaps)))
    med = [statistics.median(c) for c in zip(*rows)]
    print(f"{len(keep)} forwards of {nk} kernels on {len(by_stream)} streams (median per forward):")
    print(f"  span {med[0]:.1f} us = kernels {med[1]:.1f} + boundary gaps {med[2]:.1f} us "
          f"({100 * med[2] / med[0]:.1f} %); median gap {med[6]:.2f} us, largest {med[3]:.1f} us")
    print(f"  layer-4 tail (kernels {l4}..{nk - 1}): kernels {med[4]:.1f} us, boundary gaps {med[5]:.1f} us")
    print("  per position (median duration / median gap before it):")
    for i in range(nk):
        d = statistics.median((k[i][1] - k[i][0]) / 1e3 for k in keep)
        g = statistics.median(max(0, k[i][0] - k[i - 1][1]) / 1e3 for k in keep) if i else 0.0
        print(f"  {i:3d} {d:8.2f} {g:7.2f}  {keep[0][i][2].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0][:60]}")


if __name__ == "__main__":
    main()
