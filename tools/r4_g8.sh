#!/bin/bash
set -e
cd tools/bin
for v in base ld1 ld3 ld0 ns ent base ld1 ld0np ld0ns; do timeout -k 10 60 ./sk_$v 2048 98304 >> $GRAFT_REPO_ROOT/gpurun_out/r4_sk6.txt; done
