# In-process A/B of the conv3->conv1 chain (all boundaries / none / without the 1-block-per-CU ones).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/chain
mkdir -p $OUT
timeout -k 10 400 python3 tools/ab_bench.py --rounds 8 --steps 100 --tag chain_ab2 \
  --variants chain=1 chain=0 chain_skip=layer1.2 chain_skip=layer1.2+layer2.1+layer2.2 chain_skip=layer1.0+layer1.2 \
  > $OUT/ab2.jsonl 2> $OUT/ab2.err || { tail -20 $OUT/ab2.err; exit 1; }
cut -c1-200 $OUT/ab2.jsonl
