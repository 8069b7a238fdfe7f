# one serial forward's kernel sequence (graph replay) with durations: per-layer time map
export TMPDIR=/tmp
OUT=gpurun_out/r5seq3
mkdir -p $OUT
REGIME=serial GRAPH=1 ITERS=20 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python3 tools/probe/forward_probe.py > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
python3 - <<'PY'
import sqlite3, glob
f = glob.glob('gpurun_out/r5seq3/prof/**/*.db', recursive=True)[0]
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
python3 tools/kernel_summary.py gpurun_out/r5seq3/prof --window 900 --per 20 --top 25 > gpurun_out/r5seq3/summary.txt
head -3 gpurun_out/r5seq3/summary.txt
for t in shipped new; do
  if [ $t = shipped ]; then git_tab=tools/probe/tables/r4_serial_shipped.json; export MLS_TUNING_FILE=$git_tab; else unset MLS_TUNING_FILE; fi
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --serial --steps 100 --warmup 10 > gpurun_out/r5seq3/serial_${t}.json 2>> gpurun_out/r5seq3/err.log || { tail -20 gpurun_out/r5seq3/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5seq3/serial_${t}.json')); print('$t', 'serial', d['value'], d['ms_per_step'], d['p50_latency_ms'])"
done
