#!/bin/bash
# Round 5, calls S, T, U (tools/timek.hip variants built with the GF_EXP_* / GF_AUX_* knobs of
# this commit): uniform counts, zero-record descriptors per memory stream, last-use cache policy.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5stu.txt
cd tools/exp
for v in s0 cc ld0 ns nv nsv na nacc al a5 alp5 alp5s1 alp5n3; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O || exit 1; done
