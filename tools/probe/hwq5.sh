# 5 hardware queues for 5 slot streams (one each) vs the default 4.
export TMPDIR=/tmp
CONFIGS="GPU_MAX_HW_QUEUES=4
GPU_MAX_HW_QUEUES=5
GPU_MAX_HW_QUEUES=5 INFLIGHT=6" TAG=hwq5_s20 ROUNDS=3 STEPS=20 BENCH_ARGS="--warmup 5" bash tools/probe/proc_ab.sh || exit 1
CONFIGS="GPU_MAX_HW_QUEUES=4
GPU_MAX_HW_QUEUES=5" TAG=hwq5_s300 ROUNDS=1 STEPS=300 bash tools/probe/proc_ab.sh
