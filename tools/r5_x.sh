#!/bin/bash
# Round 5, call X: stage-1 prefetch 2 steps ahead at r <= 2 (GF_P1PFD_R2) against 1;
# tools/timek.hip r=2 and r=1 at 2048^3 (512-slice segments) and 1024^3 (one 1024-slice segment,
# config G2's geometry).
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5x.txt
cd tools/exp
for rep in 1 2; do
  for v in r2p1 r2p2 r1p1 r1p2; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O || exit 1; done
  for v in r2p1 r2p2; do timeout -k 10 90 ./tk_$v 1024 ${v}_1024 1024 >> $O || exit 1; done
done
