#!/bin/bash
# Round 5, call I: t-march stage prefetch depth (1-4 steps ahead; 1024 threads, 2 voxels each)
# against the round's first form (mz12), tools/timetshare.hip.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r5_i.txt
cd tools/exp
for v in mz12 d1 d2 d3 d4 mz12 d1 d2 d3 d4; do timeout -k 10 120 ./ts_$v 1024 $v >> $O; done
