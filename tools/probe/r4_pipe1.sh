export TMPDIR=/tmp
mkdir -p gpurun_out/pipe1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pipe_gpu.py > gpurun_out/pipe1/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/pipe1/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/pipe_probe.py > gpurun_out/pipe1/probe.jsonl 2> gpurun_out/pipe1/probe.err || { tail -20 gpurun_out/pipe1/probe.err; exit 1; }
grep '"best": true' gpurun_out/pipe1/probe.jsonl
