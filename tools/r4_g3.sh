#!/bin/bash
# round 4: 4-D three-kernel form + Gaussian LDS-DMA — tests then timings
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gaussian_gpu.py tests/test_guided_filter_gpu.py tests/test_cli_gpu.py -k "gauss or 4d or guided4d or tz_blocks or split_over or chunk_row" > gpurun_out/r4_g3_pytest.txt 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u tools/bench_ops.py --only gaussian --reps 10 >> gpurun_out/r4_gauss.jsonl 2>> gpurun_out/r4_gauss.err
  ZT_GAUSS_DMA=0 timeout -k 10 200 python -u tools/bench_ops.py --only gaussian --reps 10 >> gpurun_out/r4_gauss.jsonl 2>> gpurun_out/r4_gauss.err
done
timeout -k 10 400 python -u tools/bench_ops.py --only tshare --reps 3 --t-groups 2 4 >> gpurun_out/r4_tshare2.jsonl 2>> gpurun_out/r4_tshare2.err
ZT_G4_LEGACY=1 timeout -k 10 400 python -u tools/bench_ops.py --only tshare --reps 3 --t-groups 2 4 >> gpurun_out/r4_tshare2.jsonl 2>> gpurun_out/r4_tshare2.err
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4_tshare_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_ops.py --only tshare,gaussian --reps 2 --t-groups 2 4 > /dev/null 2>&1
cd $GRAFT_REPO_ROOT/tools/bin
for v in tk_u24 tk_seed tk_u24 tk_seed; do timeout -k 10 90 ./$v 2048 $v 512 >> $GRAFT_REPO_ROOT/gpurun_out/r4_tk2.txt; done
