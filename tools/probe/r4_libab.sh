# Same-box A/B of two builds of the kernel library (MLS_LIB_OVERRIDE): serial ResNet forward per-kernel
# profile, alternating base / new twice.  Usage: OUT=... bash tools/probe/r4_libab.sh
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/libab}
mkdir -p $OUT
run() {  # name, env...
  name=$1; shift
  env "$@" REGIME=${REGIME:-serial} GRAPH=1 ITERS=40 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -- python3 tools/probe/forward_probe.py > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; return 1; }
  python3 tools/kernel_summary.py $OUT/$name --last-of stem_pool --per 30 --top 45 > $OUT/${name}_summary.txt 2>&1
  echo "$name $(head -1 $OUT/${name}_summary.txt)"
}
run base1 MLS_LIB_OVERRIDE=$PWD/tools/probe/alt_lib/libmls_base.so && run new1 && run base2 MLS_LIB_OVERRIDE=$PWD/tools/probe/alt_lib/libmls_base.so && run new2
