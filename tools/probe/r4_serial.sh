export TMPDIR=/tmp
OUT=gpurun_out/serial
mkdir -p $OUT
run() {  # name, env...
  name=$1; shift
  env "$@" GRAPH=1 ITERS=40 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -- python3 tools/probe/forward_probe.py > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; return 1; }
  python3 tools/kernel_summary.py $OUT/$name --last-of stem_pool --per 30 --top 40 > $OUT/${name}_summary.txt 2>&1
  echo "$name $(head -1 $OUT/${name}_summary.txt)"
}
run nohead MLS_FUSED_HEAD=0 && run concurrent_table MLS_FUSED_HEAD=1 && run serial_table REGIME=serial && run serial_table_nohead REGIME=serial MLS_FUSED_HEAD=0 && run serial_table2 REGIME=serial || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_head_gpu.py tests/test_engine_gpu.py tests/test_ops_gpu.py > $OUT/head_pytest.log 2>&1; rc=$?; tail -2 $OUT/head_pytest.log
[ $rc -eq 0 ] || { grep -A30 "Error\b" $OUT/head_pytest.log | head -40; exit $rc; }
timeout -k 10 300 python3 bench.py --serial --steps 50 --warmup 10 --measure-eager 0 > $OUT/bench_serial.json 2>> $OUT/bench.err && cat $OUT/bench_serial.json
