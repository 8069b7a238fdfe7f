# End-of-session check: GPU tests, smoke, flagship bench at the driver's settings (x2) and steady
# state, a rocprofv3 kernel summary of the serial forward, and ResNet-50 over HTTP (native front end).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/final
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20_$i.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench_s20_$i.json
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 300 --warmup 20 > $OUT/bench_s300.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench_s300.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --serial --steps 20 --warmup 5 > $OUT/prof_serial.log 2>&1 || { tail -20 $OUT/prof_serial.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/kernel_summary.py $OUT/prof_serial --window 940 --per 20 --top 40 > $OUT/prof_serial_summary.txt 2>&1; head -12 $OUT/prof_serial_summary.txt
timeout -k 10 300 python3 -u tools/http_bench.py --model resnet50 --frontend native --conns 128 256 --duration 6 --warmup 2 --ready-timeout 200 > $OUT/http_resnet.jsonl 2> $OUT/http.err || { tail -20 $OUT/http.err; exit 1; }
cut -c1-330 $OUT/http_resnet.jsonl
MLS_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank.err || { tail -20 $OUT/bench_2rank.err; exit 1; }
cat $OUT/bench_2rank_gloo.json
