# Round 6: flash v2 (D = 128 transposed-O kernel) tests, then v1 / v2 timing interleaved.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_flash2}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_transformer_ops_gpu.py -x -q -k "flash" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for v in ${VERS:-1 2}; do
    MLS_FLASH_V=$v timeout -k 10 120 python3 tools/probe/flash_probe.py --batches 1 8 --tag v$v | tee -a $OUT/time.jsonl || exit 1
  done
done
