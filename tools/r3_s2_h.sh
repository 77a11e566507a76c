#!/bin/bash
# round 3 session 2, GPU call: interior tiles (mode 0) and border tiles (mode 1) as two grids on
# two streams (tk_two) vs the one mode-1 grid (base) and mode 0 over every tile (m0, bound only)
set -u
OUT=gpurun_out/r3s2h
mkdir -p $OUT
for v in base two m0 base two m0 base two; do timeout -k 10 120 tools/tk_$v 2048 $v 512 >> $OUT/tk.txt 2>&1 || { cat $OUT/tk.txt; exit 1; }; done
cat $OUT/tk.txt
