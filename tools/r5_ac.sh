#!/bin/bash
# Round 5, call AC: headline segment length (slices per workgroup march) on the final kernel
# (two-step stage-1 prefetch): 512 (product), 1024, 2048, 256; tools/timek.hip 2048^3 r=4.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5ac.txt
cd tools/exp
for rep in 1 2; do for z in 512 1024 2048 256; do timeout -k 10 90 ./tk_s0 2048 r4_zseg$z $z >> $O || exit 1; done; done
