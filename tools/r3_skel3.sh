#!/bin/bash
# Memory-only skeleton (tools/skeleton.hip, built on the CPU host) at 2048^3 r=4, one workgroup
# per CU: the product's access pattern and its ablations (loads 4 steps ahead), the streaming
# floor of a tile z-march by tile shape (TX x 2048/TX, 1 load + 1 store per voxel, with and
# without barriers), and the full pattern on 128 x 16 and 256 x 8 tiles (loads 2 steps ahead).
set -u
OUT=gpurun_out/${1:-r3skel3}
mkdir -p $OUT
for v in base nol nop3 nop5 m0l m0 m0x128 m0x256 m0x512 m0nb m0x512nb f64d2 f128d2 f256d2; do
  timeout -k 10 120 tools/sk_$v 2048 98304 >> $OUT/skeleton.txt 2>&1 || { tail -3 $OUT/skeleton.txt; exit 1; }
done
cat $OUT/skeleton.txt
