# Confirm: H2D / D2H on the slot's own stream (MLS_SLOT_COPIES=1) with launch pacing.
export TMPDIR=/tmp
CONFIGS="MLS_SLOT_COPIES=0
MLS_SLOT_COPIES=1
MLS_SLOT_COPIES=1 INFLIGHT=6
MLS_SLOT_COPIES=1 MLS_LAUNCH_PACE=0" TAG=slotcopies_s20 ROUNDS=3 STEPS=20 BENCH_ARGS="--warmup 5" bash tools/probe/proc_ab.sh || exit 1
CONFIGS="MLS_SLOT_COPIES=0
MLS_SLOT_COPIES=1" TAG=slotcopies_s300 ROUNDS=2 STEPS=300 bash tools/probe/proc_ab.sh
