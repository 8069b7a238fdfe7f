# BERT engine: CU partitions / in-flight count A/B on the current tree
export TMPDIR=/tmp
OUT=gpurun_out/r5bertpart
mkdir -p $OUT
for r in 1 2; do
  for cfg in "0 5" "2 4" "0 4" "0 6"; do
    set -- $cfg
    timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --backends fused --cu-partition $1 --inflight $2 > $OUT/p$1_i$2_$r.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    echo "part=$1 inflight=$2 run $r"; cat $OUT/p$1_i$2_$r.jsonl
  done
done
