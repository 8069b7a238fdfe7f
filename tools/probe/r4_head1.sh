export TMPDIR=/tmp
mkdir -p gpurun_out/head1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_head_gpu.py tests/test_image_decode_gpu.py > gpurun_out/head1/pytest.log 2>&1; rc=$?
tail -25 gpurun_out/head1/pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/probe/pipe_pmc.sh
