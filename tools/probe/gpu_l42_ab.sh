# A/B: shipped table vs layer4.2.conv2 on the split-K implicit GEMM (same shape/config as layer4.1.conv2)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/l42_ab.jsonl
for i in 1 2; do
timeout -k 10 200 python bench.py >> gpurun_out/l42_ab.jsonl 2>> gpurun_out/l42_ab.err || exit 1
MLS_TUNING_FILE=tools/probe/alt_tables/l42_gemm.json timeout -k 10 200 python bench.py >> gpurun_out/l42_ab.jsonl 2>> gpurun_out/l42_ab.err || exit 1
done
