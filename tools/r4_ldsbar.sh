#!/bin/bash
# 4-D box3 marches: __syncthreads() vs an LDS-only barrier (G4_LDS_BARRIER, library variant
# tools/libvar_ldsbar.so swapped in on the box copy), T share timing and 4-D parity of the variant.
set -u
O=gpurun_out/r4_ldsbar
mkdir -p $O
L=zarrs_tools_amd/libzarrs_tools_amd.so
cp $L /tmp/lib_base.so
for v in base ldsbar base ldsbar; do
  if [ $v = ldsbar ]; then cp tools/libvar_ldsbar.so $L; else cp /tmp/lib_base.so $L; fi
  timeout -k 10 300 python3 tools/bench_ops.py --only tshare --reps 5 >> $O/tshare.jsonl 2>> $O/tshare.err || exit 1
  echo "variant=$v" >> $O/tshare.jsonl
done
cp tools/libvar_ldsbar.so $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_guided_filter_gpu.py -k "4d" > $O/tests_ldsbar.txt 2>&1
cp /tmp/lib_base.so $L
echo done
