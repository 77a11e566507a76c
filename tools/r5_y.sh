#!/bin/bash
# Round 5, call Y: P3's v slices prefetched 2 steps ahead (GF_P3VPF=2, 128 VGPRs) on top of the
# two-step stage-1 prefetch (product), r = 4 f32 and u16; tools/timek.hip 2048^3.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5y.txt
cd tools/exp
for v in s0 v2 u16p2 u16v2 s0 v2 u16p2 u16v2 s0 v2; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O || exit 1; done
