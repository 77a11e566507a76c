#!/bin/bash
# round 3 session 2: output store cache policy of the fused kernel (GF_OUT_AUX: 2 = nt, product)
set -u
OUT=gpurun_out/r3s2i
mkdir -p $OUT
for v in base oa0 oa1 oa3 base oa0 oa1 oa3; do timeout -k 10 120 tools/tk_$v 2048 $v 512 >> $OUT/tk.txt 2>&1 || { cat $OUT/tk.txt; exit 1; }; done
cat $OUT/tk.txt
