# Kernel-trace one serial forward with and without the conv3->conv1 chain, plus an in-process A/B.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/chain
mkdir -p $OUT
timeout -k 10 300 python3 tools/ab_bench.py --variants chain=1 chain=0 --rounds 8 --steps 100 --tag chain_ab > $OUT/ab.jsonl 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
for c in 1 0; do
  MLS_CHAIN=$c ITERS=3 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$c -o run -- python3 tools/probe/forward_probe.py > $OUT/kt$c.log 2>&1 || { tail -20 $OUT/kt$c.log; exit 1; }
done
cat $OUT/ab.jsonl | cut -c1-220
