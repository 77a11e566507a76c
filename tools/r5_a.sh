#!/bin/bash
# Round 5, call A: persistent XCD-group schedule of the fused kernel (timek variants), times and
# L2 / fabric counters. GPU box, repo root.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r5_a.txt
cd tools/exp
for v in p0 p4 p8 p2 p16 p0 p4 p8; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O; done
cd /tmp && export TMPDIR=/tmp
for v in p0 p4 p8; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5a_tcc_$v -o run -- $GRAFT_REPO_ROOT/tools/exp/tk_$v 2048 $v 512 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5a_fetch_$v -o run -- $GRAFT_REPO_ROOT/tools/exp/tk_$v 2048 $v 512 > /dev/null 2>&1
done
echo done >> $O
