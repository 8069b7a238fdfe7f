export TMPDIR=/tmp
OUT=gpurun_out/bert4
mkdir -p $OUT
for i in 1 2; do
timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 64 128 --backends fused >> $OUT/new.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
cat $OUT/new.jsonl
