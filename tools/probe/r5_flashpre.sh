# BERT attention, 8-wave blocks: tile 1 K/V loads issued with tile 0 (MLS_FLASH_PRE=1) vs one round trip later
export TMPDIR=/tmp
OUT=gpurun_out/r5flashpre
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_models_gpu.py tests/test_e2e_gpu.py -k "flash or bert" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
  for nw in 1 0; do
    MLS_FLASH_PRE=$nw timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --backends fused > $OUT/nw${nw}_$r.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    echo "nw=$nw run $r"; cat $OUT/nw${nw}_$r.jsonl
  done
done
for nw in 1 0; do
  MLS_FLASH_PRE=$nw timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_nw$nw -o run -- python3 tools/bench_models.py bert --batches 128 --backends fused > /dev/null 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  echo "nw=$nw"; python3 -c "
import glob,csv
for f in glob.glob('$OUT/prof_nw$nw/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'flash' in r['Name'] or 'gemm_tile' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'])
" 
done
