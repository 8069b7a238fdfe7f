# Llama-3-8B 256-slot serving on the fastdiv build (base library A/B on the same box).
export TMPDIR=/tmp
OUT=gpurun_out/serve4
mkdir -p $OUT
BASE=$PWD/tools/probe/alt_lib/libmls_base.so
S="tools/bench_models.py llama-serve --batches 256 --kv-pages 769 --requests 1024 --prompt 128 --new 64"
s() {
  name=$1; shift
  env "$@" timeout -k 10 300 python3 -u $S > $OUT/$name.jsonl 2>> $OUT/serve.err || { tail -20 $OUT/serve.err; return 1; }
  echo "$name $(tail -1 $OUT/$name.jsonl)"
}
s new1 && s base1 MLS_LIB_OVERRIDE=$BASE && s new2 && s base2 MLS_LIB_OVERRIDE=$BASE
