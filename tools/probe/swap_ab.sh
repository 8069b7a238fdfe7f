# conv_gemm / halo swapped-product epilogue: numerics tests, per-call costs and bench A/B vs the
# original operand order (libmls_kernels_noswap.so, same sources built with -DMLS_CONV_SWAP=0 -DMLS_HALO_SWAP=0).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/swap2
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest tests/test_chain_gpu.py tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
NS=$GRAFT_REPO_ROOT/mlmicroservicetemplate_amd/ops/_native/libmls_kernels_noswap.so
timeout -k 10 300 python3 tools/probe/component_costs.py > $OUT/cc_swap.jsonl 2> $OUT/cc.err || { tail $OUT/cc.err; exit 1; }
MLS_LIB_OVERRIDE=$NS timeout -k 10 300 python3 tools/probe/component_costs.py > $OUT/cc_noswap.jsonl 2> $OUT/cc.err || { tail $OUT/cc.err; exit 1; }
tail -1 $OUT/cc_swap.jsonl; tail -1 $OUT/cc_noswap.jsonl
for r in 1 2; do for v in swap noswap; do
  if [ $v = noswap ]; then export MLS_LIB_OVERRIDE=$NS; else unset MLS_LIB_OVERRIDE; fi
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 > $OUT/b_${v}_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v s200 r=$r $(python3 -c "import json; d=json.load(open('$OUT/b_${v}_$r.json')); print(d['value'], d['p50_latency_ms'])")"
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/b20_${v}_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v s20 r=$r $(python3 -c "import json; d=json.load(open('$OUT/b20_${v}_$r.json')); print(d['value'], d['p50_latency_ms'])")"
done; done
