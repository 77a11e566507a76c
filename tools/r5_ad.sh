#!/bin/bash
# Round 5, call AD: the t-march with two LDS barriers per t-step (the x pass of step t + 1 in the
# interval of step t's z pass and pointwise stage; G4_TM_2BAR=1, ts_b2) against three (ts_b3),
# config T's share geometry (tools/timetshare.hip); then the 4-D GPU tests on the product library.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out
( cd tools/exp && for v in b3 b2 b3 b2 b3 b2; do timeout -k 10 120 ./ts_$v 1024 $v >> $O/r5ad.txt || exit 1; done ) || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_guided_filter_gpu.py tests/test_fullsize_gpu.py tests/test_cli_gpu.py -k "guided4d or separable_4d or t_share or tz_blocks or 4d" > $O/r5ad_tests.txt 2>&1
