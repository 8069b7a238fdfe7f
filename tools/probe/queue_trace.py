"""Which hardware queue each engine dispatch ran on, and what the early input pulls waited for.

Reads a rocprofv3 ``--kernel-trace`` CSV (Queue_Id / Stream_Id / Start / End per dispatch) of a
bench or probe run and prints, over the last ``--window`` ms of the trace:
  * per queue: its stream ids, dispatch count, busy time, and which kernel kinds ran on it;
  * per input pull (``h2d_pull_kernel``: the engine's early pull / the probe's side-stream pull):
    its queue, duration, the gap since the previous dispatch on the SAME queue ended (a pull that
    starts right as a forward kernel on its queue ends was queued behind it), and whether a forward
    kernel was running on another queue meanwhile;
  * per graph start (``h2d_pull_cell_kernel`` of the slot graph, or the stem when a graph has no
    pull): the time since the latest early pull it may depend on finished.
Usage: python tools/probe/queue_trace.py <kernel_trace.csv> [--window MS]"""
import argparse
import collections
import csv


def kind(name: str) -> str:
    if "h2d_pull_cell_kernel" in name:
        return "pull_cell"
    if "h2d_pull_kernel" in name:
        return "pull"
    for k in ("stem_pool", "head_fc", "head_finish", "conv_chain", "conv3x3", "conv_gemm"):
        if k in name:
            return k
    return name.split("(")[0].split("<")[0][-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--window", type=float, default=20.0, help="ms at the end of the trace to analyse")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                         int(r["Stream_Id"]), kind(r["Kernel_Name"]), int(r.get("Grid_Size_X") or 0)))
    rows.sort()
    t_end = max(e for _, e, *_ in rows)
    t0 = t_end - a.window * 1e6
    win = [r for r in rows if r[0] >= t0]
    print(f"{len(rows)} dispatches in the trace, {len(win)} in the last {a.window} ms")
    byq = collections.defaultdict(list)
    for r in win:
        byq[r[2]].append(r)
    for q, rs in sorted(byq.items()):
        busy = sum(e - s for s, e, *_ in rs) / 1e3
        kinds = collections.Counter(r[4] for r in rs)
        print(f"queue {q}: streams {sorted({r[3] for r in rs})}, {len(rs)} dispatches, busy {busy:.0f} us, "
              f"{dict(kinds.most_common(6))}")
    fwd = [r for r in win if r[4] not in ("pull", "pull_cell")]
    pulls = [r for r in win if r[4] == "pull"]
    print(f"\n{len(pulls)} early / side pulls (h2d_pull_kernel):")
    prev_end_q = {}
    for s, e, q, st, k, g in rows:
        if k == "pull" and s >= t0:
            before = prev_end_q.get(q)
            gap = (s - before) / 1e3 if before is not None else float("nan")
            others = sum(1 for fs, fe, fq, *_ in fwd if fq != q and fs < e and fe > s)
            print(f"  t={(s - t0) / 1e3:9.1f} us  queue {q} stream {st}  {((e - s) / 1e3):6.1f} us  "
                  f"gap after the previous dispatch on its queue {gap:7.1f} us  forward kernels overlapping on "
                  f"other queues: {others}")
        prev_end_q[q] = max(prev_end_q.get(q, 0), e)
    starts = [r for r in win if r[4] == "pull_cell"]
    if starts and pulls:
        print(f"\n{len(starts)} graph starts (h2d_pull_cell_kernel): wait since the latest early pull ended")
        for s, e, q, st, k, g in starts:
            done = [pe for ps, pe, *_ in pulls if pe <= s]
            lag = (s - max(done)) / 1e3 if done else float("nan")
            print(f"  t={(s - t0) / 1e3:9.1f} us  queue {q}  copy {((e - s) / 1e3):5.1f} us  grid {g}  "
                  f"{lag:8.1f} us after the latest pull ended")


if __name__ == "__main__":
    main()
