# Hardware queues / slot-stream copies with launch pacing on (the earlier sweeps predate pacing).
export TMPDIR=/tmp
CONFIGS="MLS_SLOT_COPIES=0
MLS_SLOT_COPIES=1
GPU_MAX_HW_QUEUES=6
GPU_MAX_HW_QUEUES=8" TAG=hwq_pace_s20 ROUNDS=2 STEPS=20 BENCH_ARGS="--warmup 5" bash tools/probe/proc_ab.sh || exit 1
CONFIGS="MLS_SLOT_COPIES=0
MLS_SLOT_COPIES=1
GPU_MAX_HW_QUEUES=8" TAG=hwq_pace_s300 ROUNDS=1 STEPS=300 bash tools/probe/proc_ab.sh
