#!/bin/bash
# Round 5, call AA: cache policy of P5's v loads (the slice's last use) on the final kernel:
# nt (aux 2) / sc1 (aux 16) against the default; tools/timek.hip 2048^3, r = 4 and r = 2.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5aa.txt
cd tools/exp
for v in s0 a5nt a5s1 r2s0 r2a5nt s0 a5nt a5s1 r2s0 r2a5nt s0 a5nt a5s1; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O || exit 1; done
