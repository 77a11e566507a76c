#!/bin/bash
# round 3, GPU call 10: fused pyramid variants (tools/timepyr) at 4096^3 u16, kernel stats + traffic
set -u
OUT=gpurun_out/r3g10
ROOT=$(pwd)
mkdir -p $OUT
timeout -k 10 180 tools/tp_pyr 4096 perlevel fused v0_65535 v1_65535 v0_64 v1_64 v1_128 v1_256 v1_16 perlevel fused > $OUT/tp.txt 2>&1 || { cat $OUT/tp.txt; exit 1; }
cat $OUT/tp.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/kt -o run --output-format csv -- $ROOT/tools/tp_pyr 4096 perlevel fused v1_64 > $ROOT/$OUT/kt.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $ROOT/$OUT/$c -o run --output-format csv -- $ROOT/tools/tp_pyr 4096 perlevel fused > $ROOT/$OUT/$c.log 2>&1 || exit 1
done
cd $ROOT
find $OUT -name "*kernel_stats.csv" | xargs cat | cut -c1-200
