#!/bin/bash
# round 3, GPU call 8: where the interior-mode split loses (single-mode launches vs the split)
set -u
OUT=gpurun_out/r3g8
mkdir -p $OUT
for v in base cur m1 m0 base cur m1 m0; do timeout -k 10 120 tools/tk_$v 2048 $v 512 >> $OUT/tk.txt 2>&1 || exit 1; done
for v in base cur m1 m0; do timeout -k 10 120 tools/tk_$v 1024 ${v}_1024 1024 >> $OUT/tk.txt 2>&1 || exit 1; done
for v in base_r2 cur_r2 m1_r2 m0_r2; do timeout -k 10 120 tools/tk_$v 1024 $v 1024 >> $OUT/tk.txt 2>&1 || exit 1; done
for v in base_r2 cur_r2 m1_r2 m0_r2; do timeout -k 10 120 tools/tk_$v 2048 ${v}_2048 256 >> $OUT/tk.txt 2>&1 || exit 1; done
cat $OUT/tk.txt
