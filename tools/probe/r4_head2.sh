export TMPDIR=/tmp
mkdir -p gpurun_out/head1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_head_gpu.py::test_resnet_fused_head_vs_unfused_and_graph > gpurun_out/head1/pytest2.log 2>&1; rc=$?
tail -5 gpurun_out/head1/pytest2.log
[ $rc -eq 0 ] || exit $rc
bash tools/probe/pipe_pmc.sh
MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/head1/bench_s20.json 2> gpurun_out/head1/bench.err || { tail -20 gpurun_out/head1/bench.err; exit 1; }
cat gpurun_out/head1/bench_s20.json
MLS_MEASURE_EAGER=0 MLS_FUSED_HEAD=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/head1/bench_s20_nohead.json 2>> gpurun_out/head1/bench.err || exit 1
cat gpurun_out/head1/bench_s20_nohead.json
