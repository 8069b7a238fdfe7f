# Pacing threshold: pace with >= N other batches in flight (default inflight - 2 = 3).
export TMPDIR=/tmp
CONFIGS="MLS_PACE_MIN_BUSY=3
MLS_PACE_MIN_BUSY=1
MLS_PACE_MIN_BUSY=2
MLS_PACE_MIN_BUSY=4" TAG=minbusy_s20 ROUNDS=3 STEPS=20 BENCH_ARGS="--warmup 5" bash tools/probe/proc_ab.sh || exit 1
CONFIGS="MLS_PACE_MIN_BUSY=3
MLS_PACE_MIN_BUSY=1" TAG=minbusy_s300 ROUNDS=1 STEPS=300 bash tools/probe/proc_ab.sh
