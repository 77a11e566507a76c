#!/bin/bash
set -e
cd tools/bin
for v in tk_u24 tk_nb1 tk_nb2 tk_nb12 tk_u24 tk_nb1 tk_nb2; do timeout -k 10 90 ./$v 2048 $v 512 >> $GRAFT_REPO_ROOT/gpurun_out/r4_tk4.txt; done
