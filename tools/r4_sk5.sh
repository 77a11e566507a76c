#!/bin/bash
set -e
cd tools/bin
for b in s4x16 s16x4 s32x2 s8x8 s16x4p32 s4x16p32 s32x2a16 s4x16 s32x2; do timeout -k 10 60 ./sk_$b 2048 98304; done
cd /tmp && export TMPDIR=/tmp
for b in s4x16 s16x4 s32x2 s32x2a16; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4pmc_$b -o run -- $GRAFT_REPO_ROOT/tools/bin/sk_$b 2048 98304 > /dev/null 2>&1
done
