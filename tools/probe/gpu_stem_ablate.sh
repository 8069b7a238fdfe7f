set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2 4 7; do
  MLS_STEM_DBG=$d timeout -k 10 200 python tools/probe/stem_pool_probe.py 2>/dev/null | sed "s/^{/{\"dbg\": $d, /" >> gpurun_out/stem_ablate.jsonl || exit 1
done
