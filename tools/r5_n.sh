#!/bin/bash
# Round 5, call N: headline kernel, LDS reads of C0 hoisted (h1: P5's before P3; h2: both phases'
# reads first, P5's arithmetic before P3's) against the product order (h0). tools/timek.hip.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r5_n.txt
cd tools/exp
for v in h0 h1 h2 h0 h1 h2; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O; done
