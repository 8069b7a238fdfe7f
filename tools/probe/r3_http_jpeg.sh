# HTTP ResNet-50 serving with JPEG uploads: the GPU image path (C++ Huffman on the
# I/O threads -> coefficient containers -> HIP IDCT/colour/resize inside the serving graph) vs the
# PIL path (GPU_IMAGE_DECODE=0, Python decode threads) vs raw RGB8 uploads.
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-http_jpeg}
mkdir -p $OUT
set -o pipefail
for io in 8 16; do
  timeout -k 10 200 python -u tools/http_bench.py --jpeg --io-threads $io --conns 128 256 --duration 6 --warmup 2 >> $OUT/http.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
timeout -k 10 200 python -u tools/http_bench.py --jpeg --jpeg-kind noise --io-threads 16 --conns 256 --duration 6 --warmup 2 >> $OUT/http.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
GPU_IMAGE_DECODE=0 timeout -k 10 200 python -u tools/http_bench.py --jpeg --io-threads 8 --decode-workers 16 --conns 256 --duration 6 --warmup 2 >> $OUT/http.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
timeout -k 10 200 python -u tools/http_bench.py --io-threads 8 --conns 256 --duration 6 --warmup 2 >> $OUT/http.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/http.jsonl
