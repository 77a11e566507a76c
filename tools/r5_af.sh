#!/bin/bash
# Round 5, call AF: t-march staging as 8-byte pairs (G4_TM_B64=1, p2) against 4-byte elements
# (b3), and the TAB stores with the nt policy (tnt, p2tnt); tools/timetshare.hip.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5af.txt
cd tools/exp
for v in b3 p2 tnt p2tnt b3 p2 tnt p2tnt; do timeout -k 10 120 ./ts_$v 1024 $v >> $O || exit 1; done
