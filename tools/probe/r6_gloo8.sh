# Round 6: 8 data-parallel ranks sharing the box's one GPU over gloo, launched both ways the driver
# can (bench.py as its own launcher, and torch.distributed.run): one JSON line from rank 0 with the
# merged per-rank layout, the process group as formed and per-rank req/s + p50.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6_gloo8
mkdir -p $OUT
MLS_DIST_BACKEND=gloo MLS_MEASURE_EAGER=0 timeout -k 10 600 python3 bench.py --gpus 8 --steps 20 --warmup 5 > $OUT/self_launch.json 2> $OUT/self.err || { tail -20 $OUT/self.err; exit 1; }
tail -1 $OUT/self_launch.json | cut -c1-2000
MLS_DIST_BACKEND=gloo MLS_MEASURE_EAGER=0 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 20 --warmup 5 > $OUT/torchrun4.json 2> $OUT/torchrun.err || { tail -20 $OUT/torchrun.err; exit 1; }
tail -1 $OUT/torchrun4.json | cut -c1-2000
