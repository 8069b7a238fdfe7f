# CU-masked slot streams (MLS_CU_PARTITION): XCD mask census, then bench variants vs the default.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/part
mkdir -p $OUT
timeout -k 10 120 python3 - > $OUT/census.txt 2>&1 <<'PY' || { cat $OUT/census.txt; exit 1; }
import torch
from mlmicroservicetemplate_amd import ops
full = ops.cu_census(torch.cuda.Stream(), blocks=4096)
print("full mask: xcc ids", sorted(set(full[:, 0].tolist())))
for layout_bits in ("roundrobin", "contiguous"):
    pass
m = ops.xcd_cu_masks()
print("xcd masks verified:", m is not None)
if m:
    print("mask0 words", [hex(w) for w in m[0]])
for lay in ("roundrobin", "contiguous"):
    for x in range(2):
        bits = [b for b in range(256) if (b % 8 if lay == "roundrobin" else b // 32) == x]
        w = [0] * 8
        for b in bits: w[b // 32] |= 1 << (b % 32)
        c = ops.cu_census(ops.cu_masked_stream(w), blocks=512)
        print(lay, x, "xcc ids", sorted(set(c[:, 0].tolist())), "distinct hw_id", len(set(c[:, 1].tolist())))
PY
cat $OUT/census.txt
run() {  # name, env..., args
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --gpus 1 $BARGS > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  echo "$name $(python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print(d['value'], d['p50_latency_ms'])")"
}
BARGS="--steps 20 --warmup 5"
run base_s20 MLS_CU_PARTITION=0
run p4_if4_s20 MLS_CU_PARTITION=4 INFLIGHT=4
run p4_if8_s20 MLS_CU_PARTITION=4 INFLIGHT=8
run p8_if8_s20 MLS_CU_PARTITION=8 INFLIGHT=8
run p4_if4_nopace_s20 MLS_CU_PARTITION=4 INFLIGHT=4 MLS_LAUNCH_PACE=0
run p2_if4_s20 MLS_CU_PARTITION=2 INFLIGHT=4
BARGS="--steps 200 --warmup 20"
run base_s200 MLS_CU_PARTITION=0
run p4_if4_s200 MLS_CU_PARTITION=4 INFLIGHT=4
run p4_if8_s200 MLS_CU_PARTITION=4 INFLIGHT=8
