export TMPDIR=/tmp
mkdir -p gpurun_out/${TAG:-gt1}
timeout -k 10 500 python -u tools/gemm_tile_probe.py ${ARGS} > gpurun_out/${TAG:-gt1}/probe.jsonl 2> gpurun_out/${TAG:-gt1}/probe.err || { tail -30 gpurun_out/${TAG:-gt1}/probe.err; exit 1; }
