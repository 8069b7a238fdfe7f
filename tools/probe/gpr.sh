#!/bin/bash
# usage: gpr.sh OUTFILE TIMEOUT 'command'   -- retries gpurun only while it reports no free box (exit 3)
out=$1; to=$2; cmd=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1; rc=$?
  if [ $rc -ne 3 ]; then echo "EXIT $rc" >> $out; exit $rc; fi
  sleep 60
done
echo "EXIT 3 (gave up)" >> $out
