# JPEG uploads over HTTP (native front end): one serving process vs WORKERS_PER_GPU processes
# sharing the port (the per-image Python decode work is GIL-bound inside one process).
OUT=$GRAFT_REPO_ROOT/gpurun_out/jpeg
mkdir -p $OUT
for cfg in "1 8" "4 4" "8 2"; do
  set -- $cfg
  timeout -k 10 300 python3 tools/http_bench.py --jpeg --workers-per-gpu $1 --decode-workers $2 --conns 64 256 --duration 8 > $OUT/b.tmp 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  sed "s/^{/{\"workers_per_gpu\": $1, \"decode_workers\": $2, /" $OUT/b.tmp | tee -a $OUT/bench.jsonl
done
