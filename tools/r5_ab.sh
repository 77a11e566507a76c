#!/bin/bash
# Round 5, call AB: config G2 geometry (1024^3 r=2) with 1024-, 512- and 256-slice segments on the
# final kernel (tools/timek.hip).
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5ab.txt
cd tools/exp
for rep in 1 2 3; do for z in 1024 512 256; do timeout -k 10 90 ./tk_r2s0 1024 r2_zseg$z $z >> $O || exit 1; done; done
