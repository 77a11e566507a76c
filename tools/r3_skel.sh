#!/bin/bash
# Memory-only skeleton of the fused guided march (tools/skeleton.hip, built on the CPU host) at
# 2048^3 r=4, one workgroup per CU (96 KiB LDS), barriers 2 per step, loads 4 steps ahead:
# the product's access pattern and ablations of it, then FETCH_SIZE / WRITE_SIZE passes.
set -u
OUT=gpurun_out/${1:-r3skel2}
ROOT=$(pwd)
mkdir -p $OUT
for v in base nol nop3 nop5 m0l m0; do
  timeout -k 10 120 tools/sk_$v 2048 98304 >> $OUT/skeleton.txt 2>&1 || { tail -3 $OUT/skeleton.txt; exit 1; }
done
cat $OUT/skeleton.txt
cd /tmp && export TMPDIR=/tmp
for v in base nol m0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c -d $ROOT/$OUT/pmc_${v}_$c -o run --output-format csv -- $ROOT/tools/sk_$v 2048 98304 > $ROOT/$OUT/pmc_${v}_$c.log 2>&1 || exit 1
  done
done
echo done
