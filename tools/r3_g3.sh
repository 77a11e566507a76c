#!/bin/bash
# round 3, GPU call 3: v3 fused kernel A/B against the round-2 kernel (timing + output compare)
set -u
OUT=gpurun_out/r3g3
mkdir -p $OUT
timeout -k 10 120 tools/tv3_r4 512 512 3 > $OUT/tv3_r4_512.txt 2>&1; rc=$?; cat $OUT/tv3_r4_512.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 tools/tv3_r4 2048 512 3 > $OUT/tv3_r4.txt 2>&1; rc=$?; cat $OUT/tv3_r4.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 tools/tv3_r2 1024 1024 3 > $OUT/tv3_r2.txt 2>&1; rc=$?; cat $OUT/tv3_r2.txt; [ $rc -eq 0 ] || exit 1
