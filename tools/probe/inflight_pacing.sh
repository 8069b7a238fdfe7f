# In-flight batches x launch pacing (on by default now): 20 and 300 steps.
export TMPDIR=/tmp
CONFIGS="INFLIGHT=5
INFLIGHT=6
INFLIGHT=8
INFLIGHT=6 MLS_LAUNCH_PACE=0" TAG=if_pace_s20 ROUNDS=2 STEPS=20 BENCH_ARGS="--warmup 5" bash tools/probe/proc_ab.sh || exit 1
CONFIGS="INFLIGHT=5
INFLIGHT=6
INFLIGHT=8" TAG=if_pace_s300 ROUNDS=2 STEPS=300 bash tools/probe/proc_ab.sh
