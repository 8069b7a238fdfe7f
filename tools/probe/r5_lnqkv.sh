# (the MLS_LN_QKV_CFG hook was probe-only and is not in ops/dispatch.py: the table cfg 15 won)
# BERT B=128: the folded QKV projection (T = 16384) on cfg 5 / 16 (c1 probe: 81.2 / 82.4 us) vs the
# table's cfg 15 (87.2 us), in the engine (5 in flight), interleaved
export TMPDIR=/tmp
OUT=gpurun_out/r5lnqkv
mkdir -p $OUT
for r in 1 2 3; do
  for c in 0 5 16; do
    if [ $c = 0 ]; then unset MLS_LN_QKV_CFG; else export MLS_LN_QKV_CFG=$c; fi
    timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 128 --backends fused > $OUT/c${c}_$r.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    echo "cfg=$c run $r $(python3 -c "import json; print(json.loads(open('$OUT/c${c}_$r.jsonl').readline())['seq_per_s'])")"
  done
done
