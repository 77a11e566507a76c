#!/bin/bash
# Round 5, call AE: price the t-march's memory streams with zero-record descriptors (outputs
# wrong): ns = no staging loads of v(t), nv = no v(tau) loads, nt = no TAB stores, nall = none;
# b3 = product. tools/timetshare.hip (t-march + box3_final on config T's share geometry).
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5ae.txt
cd tools/exp
for v in b3 ns nv nt nall b3 ns nv nt nall; do timeout -k 10 120 ./ts_$v 1024 $v >> $O || exit 1; done
