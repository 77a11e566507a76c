#!/bin/bash
# Round 5, call J: t-march with conflict-free LDS pitches (odd Vs pitch, 17-double Xs rows, lanes
# on consecutive rows in the x pass) against the first form (mz12), tools/timetshare.hip.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r5_j.txt
cd tools/exp
for v in mz12 b12 b8v2 b8 mz12 b12 b8v2 b8; do timeout -k 10 120 ./ts_$v 1024 $v >> $O; done
