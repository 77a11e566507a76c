#!/bin/bash
# Round 5, call W: stage-1 prefetch 2 steps ahead (GF_P1PFD=2) against 1 at r=3, r=5 (TY 16), u16
# r=4 and f32 r=4 (tools/timek.hip), then the GPU suite and a headline bench line on the product
# library built with it.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out
( cd tools/exp && for v in s0 p2 r3p1 r3p2 r5p1 r5p2 u16p1 u16p2 s0 p2 r3p1 r3p2 r5p1 r5p2 u16p1 u16p2; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O/r5w.txt || exit 1; done ) || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/r5w_tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline > $O/r5w_bench.json 2> $O/r5w_bench.err
