export TMPDIR=/tmp
OUT=gpurun_out/bert3
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 64 128 --backends fused > $OUT/nopart.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/nopart.jsonl
timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 64 128 --backends fused --inflight 4 --cu-partition 2 > $OUT/part.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/part.jsonl
