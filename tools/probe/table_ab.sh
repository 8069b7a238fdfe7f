# Tune full ResNet-50 tables under 1/2/3/4-way concurrency, then A/B them in bench.py at the
# driver's short run (20 steps, 5 warmup) and at steady state (300 steps), interleaved per process.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/tables
mkdir -p $OUT
for c in 1 2 3 4; do
  timeout -k 10 400 python3 -m mlmicroservicetemplate_amd.ops.autotune --concurrency $c --no-torch --out $OUT/table_c$c.json > $OUT/tune_c$c.jsonl 2> $OUT/tune_c$c.err || { tail -20 $OUT/tune_c$c.err; exit 1; }
  tail -1 $OUT/tune_c$c.jsonl
done
CONFIGS="MLS_TUNING_FILE=$GRAFT_REPO_ROOT/mlmicroservicetemplate_amd/ops/tuned/resnet50_gfx950_b32.json
MLS_TUNING_FILE=$OUT/table_c1.json
MLS_TUNING_FILE=$OUT/table_c2.json
MLS_TUNING_FILE=$OUT/table_c3.json
MLS_TUNING_FILE=$OUT/table_c4.json"
TAG=tables_s20 ROUNDS=3 STEPS=20 BENCH_ARGS="--warmup 5" CONFIGS="$CONFIGS" bash tools/probe/proc_ab.sh || exit 1
TAG=tables_s300 ROUNDS=2 STEPS=300 CONFIGS="$CONFIGS" bash tools/probe/proc_ab.sh || exit 1
