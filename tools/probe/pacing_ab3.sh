# Adaptive launch pacing (PACE x latency EWMA / inflight) vs off vs fixed 500 us.
export TMPDIR=/tmp
CONFIGS="MLS_LAUNCH_PACE=0
MLS_LAUNCH_PACE=0.9
MLS_LAUNCH_PACE=1.0
MLS_LAUNCH_GAP_US=500" TAG=pacing4_s20 ROUNDS=3 STEPS=20 BENCH_ARGS="--warmup 5" bash tools/probe/proc_ab.sh || exit 1
CONFIGS="MLS_LAUNCH_PACE=0
MLS_LAUNCH_PACE=0.9
MLS_LAUNCH_PACE=1.0" TAG=pacing4_s300 ROUNDS=2 STEPS=300 bash tools/probe/proc_ab.sh
