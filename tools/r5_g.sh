#!/bin/bash
# Round 5, call G: t-march variants (x-pass rows read from global, 2 barriers per step): tile
# depth and voxels per thread, config T's share geometry (tools/timetshare.hip).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r5_g.txt
cd tools/exp
for v in mz12 xm8 xm12 xv2 mz12 xm8 xm12 xv2; do timeout -k 10 120 ./ts_$v 1024 $v >> $O; done
