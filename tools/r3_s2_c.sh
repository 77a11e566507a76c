#!/bin/bash
# round 3 session 2, GPU call 3: block-uniform count path (tk_uni) A/B; Gaussian tile / prefetch variants
set -u
OUT=gpurun_out/r3s2c
mkdir -p $OUT
for v in base uni base uni; do timeout -k 10 120 tools/tk_$v 2048 $v 512 >> $OUT/tk.txt 2>&1 || { cat $OUT/tk.txt; exit 1; }; done
cat $OUT/tk.txt
for v in base x128 x128n1024 x128n1024p2 x128t64 x256 x128p2 t64n1024p2 basep2 x128w2 base x128 x128n1024 x128n1024p2 t64n1024p2 x256; do timeout -k 10 120 tools/tgs_$v 1024 $v >> $OUT/tgs.txt 2>&1 || { cat $OUT/tgs.txt; exit 1; }; done
cat $OUT/tgs.txt
