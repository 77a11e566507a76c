#!/bin/bash
# round 3, GPU call 6: cleaned round-2 kernel with interior mode (tk_new) vs the variants build
set -u
OUT=gpurun_out/r3g6
mkdir -p $OUT
for v in base new base new; do timeout -k 10 120 tools/tk_$v 2048 $v 512 >> $OUT/tk.txt 2>&1 || exit 1; done
for v in base_r2 new_r2 base_r2 new_r2; do timeout -k 10 120 tools/tk_$v 1024 $v 1024 >> $OUT/tk.txt 2>&1 || exit 1; done
cat $OUT/tk.txt
