#!/bin/bash
# round 3 session 2, GPU call 7: r=2 tile heights (64x32 vs 64x48) at 1024^3; Gaussian load policies
set -u
OUT=gpurun_out/r3s2f
mkdir -p $OUT
for v in r2b r2t48 r2t48k8 r2pf r2b r2t48 r2t48k8 r2pf; do timeout -k 10 120 tools/tk_$v 1024 $v 1024 >> $OUT/tk.txt 2>&1 || { cat $OUT/tk.txt; exit 1; }; done
for v in r2b r2t48 r2pf; do timeout -k 10 120 tools/tk_$v 2048 ${v}_2048 512 >> $OUT/tk.txt 2>&1 || { cat $OUT/tk.txt; exit 1; }; done
for v in base pf4 base pf4; do timeout -k 10 120 tools/tk_$v 2048 $v 512 >> $OUT/tk.txt 2>&1 || { cat $OUT/tk.txt; exit 1; }; done
cat $OUT/tk.txt
for v in x256 x256nt x256sc x256 x256nt x256sc; do timeout -k 10 120 tools/tgs_$v 1024 $v >> $OUT/tgs.txt 2>&1 || { cat $OUT/tgs.txt; exit 1; }; done
cat $OUT/tgs.txt
