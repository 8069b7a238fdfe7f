# Chain v2 (32-wide chunks: layer2 -> 3 and layer3 boundaries): numerics, then process-level A/B.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/chain2
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_chain_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
TAG=chain2_ab ROUNDS=3 STEPS=300 CONFIGS="MLS_CHAIN=1
MLS_CHAIN_SKIP=layer2.3,layer3.1,layer3.2,layer3.3,layer3.4
MLS_CHAIN_L2_CW=32
MLS_CHAIN_SKIP=layer2.3" bash tools/probe/proc_ab.sh
