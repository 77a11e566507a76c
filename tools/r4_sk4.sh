#!/bin/bash
set -e
cd tools/bin
for b in p0 px32 px16y3 px64y8 px128; do timeout -k 10 60 ./sk_$b 2048 98304; timeout -k 10 60 ./ske_$b 2048 98304; done
cd /tmp && export TMPDIR=/tmp
for b in p0 px16y3; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4pmc_$b -o run -- $GRAFT_REPO_ROOT/tools/bin/sk_$b 2048 98304 > /dev/null
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4pmcf_$b -o run -- $GRAFT_REPO_ROOT/tools/bin/sk_$b 2048 98304 > /dev/null
done
