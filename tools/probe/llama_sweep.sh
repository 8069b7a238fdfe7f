# decode-step A/B on one GPU: emulated TP=8 rank (collectives stubbed) and TP=1, at batch 1 / 8:
# skinny split cap (0 = auto, 1 = never split K across blocks) x decode chunk (64 = split +
# combine, 0 = the model's default policy).  JSON lines.
set -e
O=gpurun_out/llama_sweep.jsonl
: > $O
for tp in 8 1; do
  for ms in 0 1; do
    for ch in 64 0; do
      MLS_DEC_CHUNK=$ch timeout -k 10 200 python tools/bench_models.py llama --emulate-tp $tp --batches 1 8 --prompt 512 --steps 40 --skinny-max-split $ms 2>/dev/null | grep decode | sed "s/^{/{\"chunk\": $ch, \"ms\": $ms, /" >> $O
    done
  done
done
