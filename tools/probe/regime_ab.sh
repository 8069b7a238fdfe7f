# Under slot-stream copies: pacing factor and the layer3 chain switch, re-measured.
export TMPDIR=/tmp
CONFIGS="MLS_LAUNCH_PACE=1.0
MLS_LAUNCH_PACE=0.8
MLS_LAUNCH_PACE=1.2
MLS_CHAIN_L3=1" TAG=regime_s20 ROUNDS=3 STEPS=20 BENCH_ARGS="--warmup 5" bash tools/probe/proc_ab.sh || exit 1
CONFIGS="MLS_LAUNCH_PACE=1.0
MLS_LAUNCH_PACE=1.2
MLS_CHAIN_L3=1" TAG=regime_s300 ROUNDS=1 STEPS=300 bash tools/probe/proc_ab.sh
