#!/bin/bash
# round 3 session 2: Gaussian x pass reading its ybuf rows as 16-byte quads (GV_XQ) vs single
# floats 16 B apart (4-way LDS bank conflicts), wide and narrow tiles
set -u
OUT=gpurun_out/r3s2o
mkdir -p $OUT
for v in x256 x256xq base basexq x256 x256xq base basexq; do timeout -k 10 120 tools/tgs_$v 1024 $v >> $OUT/tgs.txt 2>&1 || { cat $OUT/tgs.txt; exit 1; }; done
cat $OUT/tgs.txt
