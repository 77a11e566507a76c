#!/bin/bash
# Round 5, call F: t-march tile depth A/B on config T's share geometry (tools/timetshare.hip).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r5_f.txt
cd tools/exp
for v in mz8 mz12 mz8 mz12; do timeout -k 10 120 ./ts_$v 1024 $v >> $O; done
