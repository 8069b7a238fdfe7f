# Clock / power under the flagship load: poll rocm-smi (timestamped) while bench.py runs ~6 s of
# steady state; bench phases are timestamped too.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/clock
mkdir -p $OUT
rm -f $OUT/smi.txt
( for i in $(seq 1 110); do echo "T $(date +%s.%N)" >> $OUT/smi.txt; rocm-smi --showclocks --showpower --json >> $OUT/smi.txt 2>/dev/null; echo >> $OUT/smi.txt; sleep 0.3; done ) &
SMI=$!
echo "start $(date +%s.%N)" > $OUT/phases.txt
MLS_BENCH_PHASES=$OUT/phases.txt timeout -k 10 150 python3 bench.py --steps 10000 --warmup 50 > $OUT/bench.log 2>&1
rc=$?
echo "end $(date +%s.%N)" >> $OUT/phases.txt
wait $SMI
cut -c1-200 $OUT/bench.log | grep metric
cat $OUT/phases.txt
python3 - <<'PY'
import json, os, re
out = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/clock")
t = None
for line in open(f"{out}/smi.txt"):
    line = line.strip()
    if line.startswith("T "):
        t = float(line[2:]); continue
    if not line.startswith("{"):
        continue
    try:
        d = json.loads(line)
    except ValueError:
        continue
    for card, v in d.items():
        if card.startswith("card"):
            print(f"{t:.2f}", v.get("sclk clock speed:"), v.get("mclk clock speed:"), v.get("fclk clock speed:"),
                  v.get("Current Socket Graphics Package Power (W)"))
PY
exit $rc
