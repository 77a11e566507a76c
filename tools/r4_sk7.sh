#!/bin/bash
# Skeleton: 64 x 16 vs 64 x 32 tiles, leaving-slice re-read at distance 9 vs 0 (is the re-read's
# cost L2 capacity?), plus TCC hit / miss passes, and the product kernel at TY = 32 vs 16. GPU box, repo root.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r4_sk7.txt
cd tools/bin
for v in t32l9 t32l0 t16l9 t16l0 t16l9s32 t16ent t32ent t32l9 t16l9; do timeout -k 10 60 ./sk_$v 2048 98304 >> $O; done
for v in tk_b32 tk_b16 tk_b32 tk_b16; do timeout -k 10 90 ./$v 2048 $v 512 >> $O; done
cd /tmp && export TMPDIR=/tmp
for v in t32l9 t16l9 t32l0 t16l0; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4pmc7_$v -o run -- $GRAFT_REPO_ROOT/tools/bin/sk_$v 2048 98304 > /dev/null 2>&1
done
echo done >> $O
