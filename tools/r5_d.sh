#!/bin/bash
# Round 5, call D: 4-D t-march stage 1 (parity tests, T-share timing + kernel trace), the fused
# mode pyramid and zarrs_ome split tests, bench.py with the extra legs.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_guided_filter_gpu.py -k "guided4d or separable_4d" tests/test_fullsize_gpu.py::test_t_share_4d_sampled_chunks > $O/r5_d_tests4d.txt 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_downsample_gpu.py tests/test_cli_gpu.py -k "gpus_split or pyramid or downsample" > $O/r5_d_tests.txt 2>&1
timeout -k 10 300 python -u tools/bench_ops.py --only tshare --reps 5 > $O/r5_d_tshare.jsonl 2> $O/r5_d_tshare.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r5_d_tshare_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_ops.py --only tshare --reps 3 > $O/r5_d_tshare_prof.log 2>&1
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 > $O/r5_d_bench.json 2> $O/r5_d_bench.err
