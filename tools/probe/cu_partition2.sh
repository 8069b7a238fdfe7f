# CU-mask layout census (which CUs a mask selects), then intra-XCD partition bench variants.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/part6
mkdir -p $OUT
timeout -k 10 120 python3 - > $OUT/census.txt 2>&1 <<'PY' || { cat $OUT/census.txt; exit 1; }
import torch, collections
from mlmicroservicetemplate_amd import ops
def show(name, w):
    c = ops.cu_census(ops.cu_masked_stream(w), blocks=4096)
    cus = ops.census_cus(c)
    per = collections.Counter(x for x, _ in cus)
    print(f"{name:28s} cus {len(cus):3d} per-xcc {dict(sorted(per.items()))} sample {sorted(cus)[:6]}")
show("full", [0xFFFFFFFF] * 8)
show("bit0", [1] + [0] * 7)
show("bits0-7", [0xFF] + [0] * 7)
show("word0", [0xFFFFFFFF] + [0] * 7)
show("word1", [0, 0xFFFFFFFF] + [0] * 6)
show("bit32", [0, 1] + [0] * 6)
show("bit1", [2] + [0] * 7)
show("xcc0 all 32 cus", [0x01010101] * 8)
for P in (2, 4, 8):  # intra-XCD
    m = ops.partition_masks(P, mode="intra")
    print("intra", P, "verified" if m else "NOT verified")
PY
cat $OUT/census.txt
run() {  # name, env..., args
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --gpus 1 $BARGS > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  echo "$name $(python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print(d['value'], d['p50_latency_ms'])") $(grep -c 'CU partitioning unavailable' $OUT/$name.err)"
}
BARGS="--steps 20 --warmup 5"
export MLS_LAUNCH_PACE=0 INFLIGHT=4
for r in 1 2; do
run p2_intra_s20_$r MLS_CU_PARTITION=2 MLS_CU_PARTITION_MODE=intra
run p2_contig_s20_$r MLS_CU_PARTITION=2 MLS_CU_PARTITION_MODE=intra_contig
done
BARGS="--steps 200 --warmup 20"
run p2_intra_s200 MLS_CU_PARTITION=2 MLS_CU_PARTITION_MODE=intra
run p2_contig_s200 MLS_CU_PARTITION=2 MLS_CU_PARTITION_MODE=intra_contig
run p4_contig_s200 MLS_CU_PARTITION=4 MLS_CU_PARTITION_MODE=intra_contig
