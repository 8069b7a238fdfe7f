# BERT-base engine throughput (5 in flight) per gemm_tile table (tools/probe/tile_tables/*.json) vs
# the shipped table and the hipBLASLt arm.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-bert_table_ab}
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python3 -u tools/bench_models.py bert --batches 32 128 --seqs 128 --steps 40 --inflight 5 --backends fused > $OUT/$name.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  sed "s/^/$name /" $OUT/$name.jsonl
}
run shipped MLS_GEMM_IMPL=native
for t in tools/probe/tile_tables/*.json; do run $(basename $t .json) MLS_GEMM_IMPL=native MLS_GEMM_TILE_TABLE=$GRAFT_REPO_ROOT/$t; done
run blas MLS_GEMM_IMPL=blas
