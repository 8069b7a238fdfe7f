# native front end with JPEG uploads (server-side PIL decode on DECODE_WORKERS threads)
set -o pipefail
mkdir -p gpurun_out
for dw in 8 16; do
  timeout -k 10 300 python -u tools/http_bench.py --model resnet50 --frontend native --jpeg --decode-workers $dw --conns 128 --duration 8 --warmup 2 >> gpurun_out/http_jpeg.jsonl 2>> gpurun_out/http_jpeg.err || exit 1
done
