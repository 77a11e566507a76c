#!/bin/bash
set -e
cd tools/bin
for v in tk_u24 tk_v5 tk_u24 tk_v5; do timeout -k 10 90 ./$v 2048 $v 512 >> $GRAFT_REPO_ROOT/gpurun_out/r4_tk5.txt; done
