#!/bin/bash
# r = 4 fused kernel with the stage-1 ring forced on (GF_P1RING_MAXR=4: 32 VGPRs spill) vs the
# product (re-reads the leaving slice). GPU box, repo root.
set -e
cd tools/bin
for v in tk_r4base tk_r4ring tk_r4base tk_r4ring; do timeout -k 10 90 ./$v 2048 $v 512 >> $GRAFT_REPO_ROOT/gpurun_out/r4_r4ring.txt; done
