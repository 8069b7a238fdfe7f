# soak: 2000-step closed-loop bench (stability of p99 / throughput over ~1.2 s of serving x 10) and a
# 60-second HTTP run at 256 connections (native front end, ResNet-50 raw uploads)
export TMPDIR=/tmp
OUT=gpurun_out/r5soak
mkdir -p $OUT
MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 2000 --warmup 20 > $OUT/s2000.json 2> $OUT/s2000.err || { tail -20 $OUT/s2000.err; exit 1; }
cat $OUT/s2000.json
timeout -k 10 300 python3 -u tools/http_bench.py --model resnet50 --frontend native --conns 256 --duration 60 --warmup 3 --ready-timeout 200 > $OUT/http60.jsonl 2> $OUT/http60.err || { tail -20 $OUT/http60.err; exit 1; }
cat $OUT/http60.jsonl
