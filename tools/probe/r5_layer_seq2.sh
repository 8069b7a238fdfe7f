# one serial forward's kernel sequence (graph replay) with durations: per-layer time map
export TMPDIR=/tmp
OUT=gpurun_out/r5seq2
mkdir -p $OUT
REGIME=serial GRAPH=1 ITERS=20 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python3 tools/probe/forward_probe.py > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
python3 - <<'PY'
import sqlite3, glob
f = glob.glob('gpurun_out/r5seq2/prof/**/*.db', recursive=True)[0]
rows = sorted(sqlite3.connect(f).execute("select start, end, name from kernels").fetchall())
# last forward: from the last stem kernel
idx = [i for i, r in enumerate(rows) if 'stem' in r[2]]
seq = rows[idx[-2]:idx[-1]]
t0 = seq[0][0]
for s, e, n in seq:
    nm = n.replace('void ', '').replace('(anonymous namespace)::', '')
    nm = nm[:nm.find('(')] if '(' in nm else nm
    print(f"{(s - t0)/1e3:8.1f} {(e - s)/1e3:7.2f}  {nm[:80]}")
PY
python3 tools/kernel_summary.py gpurun_out/r5seq2/prof --window 900 --per 20 --top 25 > gpurun_out/r5seq2/summary.txt
head -3 gpurun_out/r5seq2/summary.txt
