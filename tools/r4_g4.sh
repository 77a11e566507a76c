#!/bin/bash
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_guided_filter_gpu.py -k "4d or guided4d" > gpurun_out/r4_g4_pytest.txt 2>&1
timeout -k 10 400 python -u tools/bench_ops.py --only tshare --reps 3 --t-groups 2 4 >> gpurun_out/r4_tshare3.jsonl 2>> gpurun_out/r4_tshare3.err
cp zarrs_tools_amd/libzarrs_tools_amd.so /tmp/lib_main.so
cp tools/bin/lib_ty32.so zarrs_tools_amd/libzarrs_tools_amd.so
timeout -k 10 400 python -u tools/bench_ops.py --only tshare --reps 3 --t-groups 2 4 >> gpurun_out/r4_tshare3.jsonl 2>> gpurun_out/r4_tshare3.err
cp /tmp/lib_main.so zarrs_tools_amd/libzarrs_tools_amd.so
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4_tshare_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_ops.py --only tshare --reps 2 --t-groups 2 4 > /dev/null 2>&1
