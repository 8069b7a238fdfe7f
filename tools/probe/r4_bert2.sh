export TMPDIR=/tmp
OUT=gpurun_out/bert2
mkdir -p $OUT
for inf in 4 6; do
MLS_CU_PARTITION=2 timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 64 128 --backends fused --inflight $inf > $OUT/part_if$inf.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/part_if$inf.jsonl
done
timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 64 --backends fused > $OUT/nopart_b64.jsonl 2>> $OUT/err.log && cat $OUT/nopart_b64.jsonl
