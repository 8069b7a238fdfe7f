# in-forward tuning of the co-running (engine) table, then A/B of the result in the bench
export TMPDIR=/tmp
OUT=gpurun_out/r5inf
mkdir -p $OUT
L="layer1.0.conv1 layer2.0.conv2 layer2.0.dual layer2.1.conv1 layer3.0.conv2 layer3.0.dual layer3.1.conv1 layer3.1.conv3 layer3.2.conv1 layer3.2.conv3 layer3.3.conv1 layer3.3.conv3 layer3.4.conv1 layer3.4.conv3 layer3.5.conv1 layer3.5.conv3 layer4.0.conv1 layer4.0.conv2 layer4.0.dual layer4.1.conv1 layer4.1.conv3 layer4.2.conv1 layer4.2.conv3"
timeout -k 10 900 python3 -u tools/inforward_tune.py --regime corun --layers $L --out $OUT/corun_table.json > $OUT/corun_tune.jsonl 2> $OUT/corun_tune.err || { tail -20 $OUT/corun_tune.err; exit 1; }
head -1 $OUT/corun_tune.jsonl; tail -1 $OUT/corun_tune.jsonl
