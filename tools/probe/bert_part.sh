# BERT with partitioned engines (every sequence bucket): service GPU tests + HTTP A/B.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/bertpart
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest tests/test_service_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for P in 2 0; do
  CU_PARTITION=$P timeout -k 10 300 python3 -u tools/http_bench.py --model bert --text --frontend native --conns 64 256 --duration 6 --warmup 2 --ready-timeout 200 > $OUT/http_p$P.jsonl 2> $OUT/http_p$P.err || { tail -20 $OUT/http_p$P.err; exit 1; }
  echo "P=$P $(python3 -c "
import json
for l in open('$OUT/http_p$P.jsonl'):
    d=json.loads(l); print(d['conns'], d['requests_per_s'], d['p50_ms'], end=' | ')")"
done
