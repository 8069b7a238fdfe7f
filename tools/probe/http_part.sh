# HTTP (native front end) ResNet-50 with the partitioned engine vs CU_PARTITION=0; then the in-situ
# kernel trace of the partitioned bench.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/httppart
mkdir -p $OUT
for P in 2 0; do
  CU_PARTITION=$P timeout -k 10 300 python3 -u tools/http_bench.py --model resnet50 --frontend native --conns 128 256 --duration 6 --warmup 2 --ready-timeout 200 > $OUT/http_p$P.jsonl 2> $OUT/http_p$P.err || { tail -20 $OUT/http_p$P.err; exit 1; }
  echo "P=$P"; cut -c1-300 $OUT/http_p$P.jsonl
done
bash tools/probe/prof_partitioned.sh
