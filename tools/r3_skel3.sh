#!/bin/bash
# Streaming floor of a z-march (tools/skeleton.hip, tile only: 1 load + 1 store per voxel) by
# tile shape (TX x 2048/TX), with and without 2 barriers per step; one workgroup per CU.
set -u
OUT=gpurun_out/${1:-r3skel3}
mkdir -p $OUT
for v in m0 m0x128 m0x256 m0x512 m0nb m0x512nb; do
  for lds in 98304 0; do
    timeout -k 10 120 tools/sk_$v 2048 $lds >> $OUT/skeleton.txt 2>&1 || { tail -3 $OUT/skeleton.txt; exit 1; }
  done
done
cat $OUT/skeleton.txt
