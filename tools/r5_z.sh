#!/bin/bash
# Round 5, call Z: uniform window counts in mode-1 tiles whose apron lies inside the domain
# (GF_UNI_CNT=1; r = 4 spills 3 VGPRs) against the product, r = 4 and r = 2, tools/timek.hip 2048^3.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5z.txt
cd tools/exp
for v in s0 uc r2s0 r2uc s0 uc r2s0 r2uc; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O || exit 1; done
