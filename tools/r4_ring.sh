#!/bin/bash
# 4-D box3 marches with the z-window register ring: parity (4-D GPU tests, the full-size T share)
# then the T share timed and kernel-traced. GPU box, repo root.
set -u
O=gpurun_out/r4_ring
mkdir -p $O
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_guided_filter_gpu.py tests/test_fullsize_gpu.py tests/test_cli_gpu.py \
  -k "4d or chunk_row_grouping or t_share or tz_blocks" > $O/tests.txt 2>&1 || { echo tests failed; exit 1; }
for ring in 1 0 1 0; do
  ZT_G4_FINAL_RING=$ring timeout -k 10 300 python3 tools/bench_ops.py --only tshare --reps 5 >> $O/tshare.jsonl 2>> $O/tshare.err || exit 1
  echo "ring=$ring" >> $O/tshare.jsonl
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/kt -o run --output-format csv -- python3 $ROOT/tools/bench_ops.py --only tshare --reps 3 > $ROOT/$O/kt.jsonl 2>&1 ) || exit 1
echo done
