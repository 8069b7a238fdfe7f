# Halo kernel: skip the all-padding row blocks (MLS_HALO_SKIP_PAD) -- numerics, per-call costs, bench A/B.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/skip
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest tests/test_ops_gpu.py -k "halo or resnet or e2e" tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
NS=$GRAFT_REPO_ROOT/mlmicroservicetemplate_amd/ops/_native/libmls_kernels_noskip.so
timeout -k 10 300 python3 tools/probe/component_costs.py > $OUT/cc_skip.jsonl 2> $OUT/cc.err || { tail $OUT/cc.err; exit 1; }
MLS_LIB_OVERRIDE=$NS timeout -k 10 300 python3 tools/probe/component_costs.py > $OUT/cc_noskip.jsonl 2> $OUT/cc.err || { tail $OUT/cc.err; exit 1; }
tail -1 $OUT/cc_skip.jsonl; tail -1 $OUT/cc_noskip.jsonl
for r in 1 2; do for v in skip noskip; do
  if [ $v = noskip ]; then export MLS_LIB_OVERRIDE=$NS; else unset MLS_LIB_OVERRIDE; fi
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 > $OUT/b_${v}_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$v s200 r=$r $(python3 -c "import json; d=json.load(open('$OUT/b_${v}_$r.json')); print(d['value'], d['p50_latency_ms'])")"
done; done
