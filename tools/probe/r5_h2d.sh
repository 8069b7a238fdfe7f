export TMPDIR=/tmp
mkdir -p gpurun_out/r5h2d
timeout -k 10 120 python3 tools/probe/h2d_pull_probe.py > gpurun_out/r5h2d/pull.json 2>&1; cat gpurun_out/r5h2d/pull.json
MLS_STEM_RAWBAR=0 timeout -k 10 120 python3 tools/probe/stem_pool_probe.py 2>&1 | grep concurrency
MLS_STEM_RAWBAR=1 timeout -k 10 120 python3 tools/probe/stem_pool_probe.py 2>&1 | grep concurrency
