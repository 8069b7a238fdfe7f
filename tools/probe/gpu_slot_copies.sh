# copies on the shared H2D/D2H streams vs on each slot's compute stream, at 5 and 8 in flight
set -o pipefail
mkdir -p gpurun_out
for n in 5 8; do
  timeout -k 10 200 python bench.py --inflight $n --steps 400 --warmup 40 > gpurun_out/bench_sc0_$n.log 2>&1 || exit 1
  MLS_SLOT_COPIES=1 timeout -k 10 200 python bench.py --inflight $n --steps 400 --warmup 40 > gpurun_out/bench_sc1_$n.log 2>&1 || exit 1
done
