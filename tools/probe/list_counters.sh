export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
grep -oE "^[[:space:]]*(SQ|TCC|TCP|GRBM|TA|TD|SPI)[A-Z0-9_]*" $OUT/counters_list.txt | sort -u | head -400 > $OUT/counter_names.txt || true
wc -l $OUT/counter_names.txt
