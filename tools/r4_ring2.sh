#!/bin/bash
# box3_final ring form: 64 x 16 vs 64 x 32 output tiles (ZT_G4_FINAL_TY), parity of both, timing.
set -u
O=gpurun_out/r4_ring2
mkdir -p $O
for ty in 16 32; do
  ZT_G4_FINAL_TY=$ty timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_guided_filter_gpu.py tests/test_fullsize_gpu.py \
    -k "4d or chunk_row_grouping or t_share" > $O/tests_ty$ty.txt 2>&1 || { echo tests failed; exit 1; }
done
for ty in 16 32 16 32; do
  ZT_G4_FINAL_TY=$ty timeout -k 10 300 python3 tools/bench_ops.py --only tshare --reps 5 >> $O/tshare.jsonl 2>> $O/tshare.err || exit 1
  echo "ty=$ty" >> $O/tshare.jsonl
done
echo done
