#!/bin/bash
# Skeleton: leaving slice re-read from the array (distance 9) vs from a per-workgroup ring buffer
# of the entering quads in global memory (coalesced), with and without the P3/P5 reloads; TCC
# passes. Binaries in tools/exp (built in the container). GPU box, repo root.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r4_rb.txt
cd tools/exp
for v in rb0 rb1 rb0np rb1np ld0np rb0 rb1; do timeout -k 10 60 ./sk_$v 2048 98304 >> $O; done
cd /tmp && export TMPDIR=/tmp
for v in rb0 rb1; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4pmcrb_$v -o run -- $GRAFT_REPO_ROOT/tools/exp/sk_$v 2048 98304 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4pmcrbf_$v -o run -- $GRAFT_REPO_ROOT/tools/exp/sk_$v 2048 98304 > /dev/null 2>&1
done
echo done >> $O
