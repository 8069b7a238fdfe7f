# Native staging pool vs Python copy threads: host copy rate, then interleaved bench.py A/B at the
# driver's settings (20 steps, warmup 5) and one steady-state (300 steps) pair.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/staging_ab
mkdir -p $OUT
timeout -k 10 120 python3 tools/probe/staging_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -5 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
CONFIGS="MLS_NATIVE_STAGING=1
MLS_NATIVE_STAGING=0
MLS_NATIVE_STAGING=1 MLS_STAGE_THREADS=8" TAG=staging_ab ROUNDS=3 STEPS=20 BENCH_ARGS="--warmup 5" bash tools/probe/proc_ab.sh || exit 1
CONFIGS="MLS_NATIVE_STAGING=1
MLS_NATIVE_STAGING=0" TAG=staging_ab_s300 ROUNDS=1 STEPS=300 bash tools/probe/proc_ab.sh
