#!/bin/bash
# Round 5, call E: the t-march stage 1 with buffer accesses and LDS-only barriers: 4-D parity
# tests (incl. the full-size T share), T-share timing and kernel trace.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_guided_filter_gpu.py tests/test_fullsize_gpu.py -k "guided4d or separable_4d or t_share" > $O/r5_e_tests4d.txt 2>&1
timeout -k 10 300 python -u tools/bench_ops.py --only tshare --reps 5 > $O/r5_e_tshare.jsonl 2> $O/r5_e_tshare.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r5_e_tshare_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_ops.py --only tshare --reps 3 > $O/r5_e_tshare_prof.log 2>&1
