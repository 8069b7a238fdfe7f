# Deep-ring conv_gemm configs (19, 23..28) vs the shipped table's picks on the latency-bound
# layer3 / layer4 layers, under 4-way concurrency (the tuner's scoring), after their numerics tests.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/deepring
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_ops_gpu.py -x -q -k "resnet_shapes or stem or test_gemm" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python3 -m mlmicroservicetemplate_amd.ops.autotune --concurrency 4 --no-torch \
  --layers layer2.0.conv2 layer3.0.conv1 layer3.0.conv2 layer3.1.conv1 layer3.1.conv3 layer3.0.dual \
           layer4.0.conv1 layer4.0.conv2 layer4.1.conv1 layer4.1.conv2 layer4.1.conv3 layer4.0.dual \
  --cfgs 4 7 8 9 10 12 14 19 23 24 25 26 27 28 > $OUT/tune_c4.jsonl 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
cat $OUT/tune_c4.jsonl | cut -c1-200
