# Hardware queues per process vs in-flight batches with the final kernels.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/hwq.jsonl
for q in 6 8; do
  for n in 5 6 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --inflight $n --steps 400 --warmup 40 2>/dev/null | sed "s/^{/{\"hw_queues\": $q, /" >> gpurun_out/hwq.jsonl || exit 1
  done
done
