# Engine GPU tests with the partitioned default, bench default, HW-queue variants, BERT partition A/B.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/t1
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gpu.py tests/test_e2e_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
run() {  # name, env..., args
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --gpus 1 $BARGS > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  echo "$name $(python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print(d['value'], d['p50_latency_ms'], d['config']['inflight'], d['config']['cu_partitions'])")"
}
BARGS="--steps 20 --warmup 5"
run default_s20_1
run hwq6_if6_s20 GPU_MAX_HW_QUEUES=6 MLS_HW_QUEUES=6 INFLIGHT=6
run hwq8_if8_s20 GPU_MAX_HW_QUEUES=8 MLS_HW_QUEUES=8 INFLIGHT=8
run default_s20_2
BARGS="--steps 200 --warmup 20"
run default_s200
run hwq6_if6_s200 GPU_MAX_HW_QUEUES=6 MLS_HW_QUEUES=6 INFLIGHT=6
for P in 0 2; do
  MLS_CU_PARTITION=$P timeout -k 10 300 python3 tools/bench_models.py bert --batches 32 128 --backends fused --steps 60 > $OUT/bert_p$P.jsonl 2> $OUT/bert_p$P.err || { tail -20 $OUT/bert_p$P.err; exit 1; }
  cat $OUT/bert_p$P.jsonl
done
