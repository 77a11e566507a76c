#!/bin/bash
# round 3 session 2: r=2 at 8 waves per SIMD (two 1024-thread workgroups per CU, 64 VGPRs, 25
# spilled) vs the product (4 waves per SIMD), 1024^3 with 1024- and 512-slice segments
set -u
OUT=gpurun_out/r3s2m
mkdir -p $OUT
for v in r2b:1024 r2w8:1024 r2w8:512 r2b:512 r2b:1024 r2w8:1024 r2w8:512; do timeout -k 10 120 tools/tk_${v%%:*} 1024 $v ${v#*:} >> $OUT/tk.txt 2>&1 || { cat $OUT/tk.txt; exit 1; }; done
cat $OUT/tk.txt
