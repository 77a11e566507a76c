#!/bin/bash
# round 3 session 2, GPU call 4: wide-tile Gaussian variants (tools/timegauss.hip)
set -u
OUT=gpurun_out/r3s2d
mkdir -p $OUT
for v in base x256 x256t24 x256t24p2 x256t28 x192 x192t24p2 x128t64 base x256 x256t24 x256t24p2 x256t28 x192 x192t24p2 x128t64; do timeout -k 10 120 tools/tgs_$v 1024 $v >> $OUT/tgs.txt 2>&1 || { cat $OUT/tgs.txt; exit 1; }; done
cat $OUT/tgs.txt
