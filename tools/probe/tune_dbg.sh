export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/tunedbg
mkdir -p $OUT
timeout -k 10 200 python3 -X faulthandler -u -m mlmicroservicetemplate_amd.ops.autotune --batch 32 --concurrency 4 --no-torch --layers layer3.1.conv1 > $OUT/plain.log 2>&1; echo "plain rc $?"; tail -3 $OUT/plain.log
MLS_TUNE_PARTITIONS=2 timeout -k 10 200 python3 -X faulthandler -u -m mlmicroservicetemplate_amd.ops.autotune --batch 32 --concurrency 4 --no-torch --layers layer3.1.conv1 > $OUT/part.log 2>&1; echo "part rc $?"; tail -30 $OUT/part.log
