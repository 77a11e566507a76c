#!/bin/bash
# Round 5, call B: persistent schedule + loose lockstep (lead bound GF_LOCK steps), A/B times
# and L2 / fabric counters. GPU box, repo root.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r5_b.txt
cd tools/exp
for v in p0 p4 l4s2 l4s4 l4s8 l8s4 l2s4 l16s4 p0 l4s2 l4s4; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O; done
cd /tmp && export TMPDIR=/tmp
for v in l4s2 l4s4; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5b_tcc_$v -o run -- $GRAFT_REPO_ROOT/tools/exp/tk_$v 2048 $v 512 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5b_fetch_$v -o run -- $GRAFT_REPO_ROOT/tools/exp/tk_$v 2048 $v 512 > /dev/null 2>&1
done
echo done >> $O
