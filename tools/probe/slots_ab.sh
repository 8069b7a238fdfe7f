# Partitioned engine: extra slots sharing the masked streams (6 slots / 4 streams) with H2D / D2H
# on the shared copy streams (MLS_SLOT_COPIES=0) so a stream-mate's batch is staged and copied in
# while the stream computes.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/slots
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --gpus 1 $BARGS > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  echo "$name $(python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print(d['value'], d['p50_latency_ms'], d['config']['inflight'])")"
}
for r in 1 2; do
BARGS="--steps 200 --warmup 20"
run A_s200_$r
run B_if6_copies0_s200_$r INFLIGHT=6 MLS_SLOT_COPIES=0
run C_if6_s200_$r INFLIGHT=6
run D_if4_copies0_s200_$r MLS_SLOT_COPIES=0
BARGS="--steps 20 --warmup 5"
run A_s20_$r
run B_if6_copies0_s20_$r INFLIGHT=6 MLS_SLOT_COPIES=0
done
