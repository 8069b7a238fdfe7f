# LayerNorm kernel time, base vs new library, in the BERT B=128 forward (rocprofv3 kernel trace).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/lnprof
mkdir -p $OUT
p() {
  name=$1; shift
  cd /tmp && env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run -- python3 $R/tools/bench_models.py bert --batches 128 --inflight 1 --steps 10 --backends fused > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; return 1; }
  cd $R && python3 tools/kernel_summary.py $OUT/$name --window 4000 --per 10 --top 6 > $OUT/${name}_summary.txt 2>&1
  echo "$name"; cat $OUT/${name}_summary.txt
}
p base MLS_LIB_OVERRIDE=$R/tools/probe/alt_lib/libmls_base.so && p new
