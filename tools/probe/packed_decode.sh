# Packed-weight decode GEMMs: numerics, cold-stream probe of the launch variants (M = 1 and 8),
# and the Llama-3-8B TP=1 decode bench with the packed path off / on / on without the residual
# fold (MLS_PACKED_DECODE, MLS_PACKED_FOLD).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/packed
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_skinny_packed_gpu.py tests/test_llama_tp_gpu.py > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
for m in ${PROBE_M:-1 8}; do
  M=$m PACKED_VARIANTS=${PACKED_VARIANTS:-9,25,10,11,12,13} timeout -k 10 300 python3 -u tools/decode_stream_probe.py > $OUT/probe_m$m.jsonl 2>$OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
done
for cfg in "MLS_PACKED_DECODE=0" "MLS_PACKED_FOLD=0" "MLS_PACKED_FOLD=1" ${EXTRA_CFGS}; do
  env $cfg timeout -k 10 300 python3 tools/bench_models.py llama --batches 1 4 8 16 --steps 30 > $OUT/bench.tmp 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  sed "s/^{/{\"cfg\": \"$cfg\", /" $OUT/bench.tmp | tee -a $OUT/bench.jsonl
done
