# In-flight sweep with the final kernels (throughput vs p50).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/inflight2.jsonl
for n in 3 4 5 6 8; do
  timeout -k 10 200 python bench.py --inflight $n --steps 400 --warmup 40 >> gpurun_out/inflight2.jsonl 2>/dev/null || exit 1
done
