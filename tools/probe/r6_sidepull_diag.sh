# Which part of the side-stream pull arm is slow untraced: its cross-stream event waits (SYNC=event),
# nothing (SYNC=none, timing only), or the pull itself as an extra launch on the slot stream (SYNC=same)
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6_sidepull; mkdir -p $OUT
for sync in event none same; do
  for side in masked plain; do
    [ $sync = same ] && [ $side = plain ] && continue
    echo "== SYNC=$sync SIDE=$side" | tee -a $OUT/diag.txt
    SYNC=$sync SIDE=$side timeout -k 10 180 python3 tools/probe/engine_gap_probe.py >> $OUT/diag.txt 2>&1 || { tail -20 $OUT/diag.txt; exit 1; }
    tail -3 $OUT/diag.txt
  done
done
