# 4 data-parallel ranks sharing the box's one GPU over gloo (the driver's N=4 path with RCCL on
# 4 GPUs runs the same code): one JSON line from rank 0, value = whole-job req/s.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/gloo4
mkdir -p $OUT
MLS_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/bench.json
