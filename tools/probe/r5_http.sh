# HTTP serving on the round-5 tree (native front end): ResNet-50 raw RGB8 and JPEG uploads, BERT text
export TMPDIR=/tmp
OUT=gpurun_out/r5http
mkdir -p $OUT
hb() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python3 -u tools/http_bench.py "$@" --frontend native --duration 6 --warmup 2 --ready-timeout 200 > $OUT/$name.jsonl 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  echo "$name $(python3 -c "
import json
for l in open('$OUT/$name.jsonl'):
    d=json.loads(l); print(d['conns'], d['requests_per_s'], d['p50_ms'], end=' | ')")"
}
hb resnet_raw --model resnet50 --conns 128 256
hb resnet_jpeg --model resnet50 --jpeg --conns 128 256
hb bert_text --model bert --text --conns 128 256
