#!/bin/bash
# Round 5, call Q: t-march x / y pass items of 4, 8, 16 outputs (tools/timetshare.hip, config T's
# share geometry), then the LDS-array occupancy of the headline kernel (SQ_LDS_IDX_ACTIVE & co.).
set -u
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O/r5q
( cd tools/exp && for v in k44 k84 k88 k168 k44 k84 k88 k168; do timeout -k 10 120 ./ts_$v 1024 $v >> $O/r5q/tmarch_k.txt || exit 1; done ) || exit 1
PASSES="lds" tools/profile_pmc.sh gpurun_out/r5q --steps 1 --warmup 0 --parity-chunks 0 || exit 1
python3 tools/pmc_summary.py gpurun_out/r5q gf3d $((2048*2048*2048)) > gpurun_out/r5q/summary.txt
