#!/bin/bash
# Round 5, call AM: idle waves not branching around P4 (GF_WAVE_SKIP=0) at r = 4 f32, r = 2 f32
# (2048^3 and G2's 1024^3) and r = 4 u16; tools/timek.hip.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5am.txt
cd tools/exp
for rep in 1 2 3; do
  for v in s0 ws0 r2s0 r2ws0 u16s0 u16ws0; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O || exit 1; done
  for v in r2s0 r2ws0; do timeout -k 10 90 ./tk_$v 1024 ${v}_1024 1024 >> $O || exit 1; done
done
