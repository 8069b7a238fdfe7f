# Re-tune the layers whose in-forward time exceeds their tuned time (unchained 1x1 convs, the duals,
# the stride-2 3x3s: tools/probe/r5_layer_seq.sh) with the L2 flushed between timed calls
# (MLS_TUNE_FLUSH_MB), in the serial and the engine (4 copies on 2 CU-masked halves) regimes
export TMPDIR=/tmp
OUT=gpurun_out/r5flushtune
mkdir -p $OUT
L="layer1.0.conv1 layer2.1.conv1 layer3.1.conv1 layer3.2.conv1 layer3.3.conv1 layer3.4.conv1 layer3.5.conv1 layer3.1.conv3 layer3.2.conv3 layer3.3.conv3 layer3.4.conv3 layer3.5.conv3 layer4.0.conv1 layer4.1.conv1 layer4.2.conv1 layer4.1.conv3 layer4.2.conv3 layer2.0.dual layer3.0.dual layer4.0.dual layer2.0.conv2 layer3.0.conv2 layer4.0.conv2"
MLS_TUNE_FLUSH_MB=64 timeout -k 10 540 python3 -u -m mlmicroservicetemplate_amd.ops.autotune --concurrency 1 --no-torch --layers $L --out $OUT/serial_flush.json > $OUT/serial.jsonl 2> $OUT/serial.err || { tail -20 $OUT/serial.err; exit 1; }
tail -1 $OUT/serial.jsonl
MLS_TUNE_FLUSH_MB=64 MLS_TUNE_PARTITIONS=2 timeout -k 10 600 python3 -u -m mlmicroservicetemplate_amd.ops.autotune --concurrency 4 --no-torch --layers $L --out $OUT/conc_flush.json > $OUT/conc.jsonl 2> $OUT/conc.err || { tail -20 $OUT/conc.err; exit 1; }
tail -1 $OUT/conc.jsonl
