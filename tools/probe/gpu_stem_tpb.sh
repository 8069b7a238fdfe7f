# Fused stem kernel: tiles per block sweep (numerics for each, then graph-timed per call), then
# the ablation flags at the default tiles per block.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/stem_tpb.jsonl
for t in 1 2 4 7; do
  MLS_STEM_TPB=$t timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "stem" > gpurun_out/stem_test_tpb$t.log 2>&1 || exit 1
  MLS_STEM_TPB=$t timeout -k 10 200 python tools/probe/stem_pool_probe.py 2>/dev/null | sed "s/^{/{\"tpb\": $t, /" >> gpurun_out/stem_tpb.jsonl || exit 1
done
for d in 1 2 4 7; do
  MLS_STEM_DBG=$d timeout -k 10 200 python tools/probe/stem_pool_probe.py 2>/dev/null | sed "s/^{/{\"tpb\": 4, \"dbg\": $d, /" >> gpurun_out/stem_tpb.jsonl || exit 1
done
