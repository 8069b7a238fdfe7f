# bench.py in-flight batches sweep (concurrent per-slot streams), default and 8 HW queues
set -o pipefail
mkdir -p gpurun_out
for n in 5 6 8 12; do
  timeout -k 10 200 python bench.py --inflight $n --steps 400 --warmup 40 > gpurun_out/bench_inflight_$n.log 2>&1 || exit 1
done
for n in 6 8; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --inflight $n --steps 400 --warmup 40 > gpurun_out/bench_inflight_${n}_q8.log 2>&1 || exit 1
done
