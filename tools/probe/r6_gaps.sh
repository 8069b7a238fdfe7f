# Kernel-boundary cost of the ResNet-50 forward (tools/probe/boundary_gaps.py), co-running bench and
# serial bench, from rocprofv3 kernel traces.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_gaps}
mkdir -p $OUT
cd $R
for arm in corun serial; do
  extra=""; [ $arm = serial ] && extra="--serial"
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$arm -o run -- python3 bench.py --steps 120 --warmup 10 --measure-eager 0 $extra > $OUT/$arm.json 2> $OUT/$arm.err || { tail -20 $OUT/$arm.err; exit 1; }
  f=$(find $OUT/prof_$arm -name "*kernel_trace.csv" | head -1)
  python3 tools/probe/boundary_gaps.py "$f" > $OUT/gaps_$arm.txt || exit 1
  gzip -c "$f" > $OUT/trace_$arm.csv.gz; rm -rf $OUT/prof_$arm
  head -4 $OUT/gaps_$arm.txt
done
