#!/bin/bash
# Round 5, call H: t-march with the LDS stage + Markstein count divisions, fast a = s/(s+eps),
# running U4: tile depth / voxels per thread A/B (tools/timetshare.hip).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r5_h.txt
cd tools/exp
for v in mz12 em8 em12 ev2 mz12 em8 em12 ev2; do timeout -k 10 120 ./ts_$v 1024 $v >> $O; done
