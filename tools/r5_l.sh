#!/bin/bash
# Round 5, call L: the final t-march form (product defaults) against mz12; 4-D parity tests;
# device-resident mode pyramid (zarrs_ome --discrete) and mean pyramid timings with a kernel trace.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
cd tools/exp
for v in fin mz12 fin mz12; do timeout -k 10 120 ./ts_$v 1024 $v >> $O/r5_l.txt; done
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_guided_filter_gpu.py tests/test_fullsize_gpu.py tests/test_downsample_gpu.py -k "guided4d or separable_4d or t_share or pyramid or mode" > $O/r5_l_tests.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r5_l_pyr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_ops.py --only pyramid,pyramid_discrete,tshare --reps 5 > $O/r5_l_ops.jsonl 2> $O/r5_l_ops.err
