export TMPDIR=/tmp
OUT=gpurun_out/serial2
mkdir -p $OUT
run() {  # name, env...
  name=$1; shift
  env "$@" GRAPH=1 ITERS=40 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -- python3 tools/probe/forward_probe.py > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; return 1; }
  python3 tools/kernel_summary.py $OUT/$name --last-of stem_pool --per 30 --top 45 > $OUT/${name}_summary.txt 2>&1
  echo "$name $(head -1 $OUT/${name}_summary.txt)"
}
run serial_shipped REGIME=serial && run serial_retune MLS_TUNING_FILE=tools/probe/alt_tables/resnet50_r4_serial_retune.json && run serial_shipped2 REGIME=serial && run serial_retune2 MLS_TUNING_FILE=tools/probe/alt_tables/resnet50_r4_serial_retune.json
