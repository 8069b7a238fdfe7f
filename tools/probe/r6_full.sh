# Round 6: the whole GPU suite (as the driver runs it), then the Llama-3-8B TP=1 numbers on native routes.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6_full
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
