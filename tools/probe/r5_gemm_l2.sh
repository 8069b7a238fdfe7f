# L2 hit rate of the tile GEMM (cfg 15) vs hipBLASLt on sq8k / BERT FFN-up: what the loads cost
export TMPDIR=/tmp
OUT=gpurun_out/r5l2
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $OUT/pmc -o run -- python3 tools/gemm_tile_probe.py --shapes sq8k bert128_ffn1 --cfgs 15 --conc 1 --iters 3 > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
python3 - <<'PY'
import sqlite3, glob, collections
f = glob.glob('gpurun_out/r5l2/pmc/**/*.db', recursive=True)[0]
c = sqlite3.connect(f)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print([t for t in tabs if 'pmc' in t.lower() or 'counter' in t.lower()][:10])
PY
