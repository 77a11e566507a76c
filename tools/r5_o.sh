#!/bin/bash
# Round 5, call O: box3_final with buffer accesses and LDS-only step barriers (bf: v loaded with
# the step's outputs; bf2: v loaded before the TAB prefetch) against the round's first form (fin),
# config T's share geometry (tools/timetshare.hip); then the 4-D parity tests on the product
# library (which carries bf2).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
cd tools/exp
for v in fin bf bf2 fin bf bf2; do timeout -k 10 120 ./ts_$v 1024 $v >> $O/r5_o.txt; done
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_guided_filter_gpu.py tests/test_fullsize_gpu.py tests/test_cli_gpu.py -k "guided4d or separable_4d or t_share or tz_blocks or 4d" > $O/r5_o_tests.txt 2>&1
