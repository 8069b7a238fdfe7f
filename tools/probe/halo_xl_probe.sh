# XL halo tile (CFG_HALO_XL) numerics + per-layer timing vs the shipped picks, alone and 4-way co-running.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/haloxl
mkdir -p $OUT
#timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py -x -q -k "halo" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
#tail -2
for c in 4 1; do
MLS_TUNE_VERBOSE=1 timeout -k 10 300 python3 -m mlmicroservicetemplate_amd.ops.autotune --concurrency $c --no-torch \
  --layers layer1.1.conv2 layer2.1.conv2 layer3.1.conv2 layer4.1.conv2 --cfgs 8 9 12 > $OUT/tune_c$c.jsonl 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
echo "c$c"; python3 -c "import json,sys; [print(d[\"layer\"], {k:v for k,v in d.get(\"tried_us\",{}).items() if k.startswith(\"10\") or k in (\"9,1\",\"12,1\",\"8,1\",\"8,2\")}) for d in map(json.loads, open(sys.argv[1])) if \"layer\" in d]" $OUT/tune_c$c.jsonl
done
