#!/bin/bash
# Round 5, call R: LLVM scheduling strategies (-mllvm -amdgpu-sched-strategy=max-ilp /
# iterative-ilp / max-memory-clause, -amdgpu-schedule-metric-bias=0) on the headline kernel
# (tools/timek.hip, 2048^3 r=4, 512-slice segments) and the t-march (tools/timetshare.hip).
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5r.txt
cd tools/exp
for v in s0 ilp iilp mc b0 s0 ilp iilp mc b0; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O || exit 1; done
for v in k44 ilp iilp k44 ilp iilp; do timeout -k 10 120 ./ts_$v 1024 ts_$v >> $O || exit 1; done
