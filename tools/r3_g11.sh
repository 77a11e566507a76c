#!/bin/bash
# round 3, GPU call 11: the 4096^3 pyramid through the library, fused vs per-level, kernel traces
set -u
OUT=gpurun_out/r3g11
ROOT=$(pwd)
mkdir -p $OUT
timeout -k 10 120 tools/tp_pyr 4096 perlevel fused > $OUT/tp.txt 2>&1 || { cat $OUT/tp.txt; exit 1; }
cat $OUT/tp.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/kt_fused -o run --output-format csv -- python3 $ROOT/tools/bench_pyramid.py --size 4096 > $ROOT/$OUT/pyr_fused.json 2>&1 || exit 1
ZT_PYRAMID_UNFUSED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/kt_unfused -o run --output-format csv -- python3 $ROOT/tools/bench_pyramid.py --size 4096 > $ROOT/$OUT/pyr_unfused.json 2>&1 || exit 1
cd $ROOT
grep '^{' $OUT/pyr_fused.json | cut -c1-400; grep '^{' $OUT/pyr_unfused.json | cut -c1-400
for k in kt_fused kt_unfused; do find $OUT/$k -name "*kernel_stats.csv" | xargs cat | cut -c1-220; done
