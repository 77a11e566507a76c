#!/bin/bash
set -e
df -h /tmp $GRAFT_REPO_ROOT > gpurun_out/r4_df.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cli_gpu.py tests/test_guided_filter_gpu.py -k "ome or 4d or guided4d or tz_blocks" > gpurun_out/r4_g6_pytest.txt 2>&1
timeout -k 10 400 python -u tools/bench_ops.py --only tshare --reps 3 --t-groups 2 4 >> gpurun_out/r4_tshare4.jsonl 2>> gpurun_out/r4_tshare4.err
ZT_G4_QUAD=0 timeout -k 10 400 python -u tools/bench_ops.py --only tshare --reps 3 --t-groups 2 4 >> gpurun_out/r4_tshare4.jsonl 2>> gpurun_out/r4_tshare4.err
timeout -k 10 900 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 4 > gpurun_out/r4_ome_e2e2.json 2> gpurun_out/r4_ome_e2e2.err
timeout -k 10 900 python -u tools/bench_e2e.py --t 32 --size 512 --radius 2 --repeat 1 --cpu-chunks 16 > gpurun_out/r4_e2e_t32_512.json 2> gpurun_out/r4_e2e_t32.err
timeout -k 10 900 python -u tools/bench_e2e.py --t 32 --size 512 --radius 2 --repeat 1 --procs 4 --check 1 > gpurun_out/r4_e2e_t32_512_p4.json 2>> gpurun_out/r4_e2e_t32.err
cd $GRAFT_REPO_ROOT/tools/bin
for v in tk_u24 tk_seed tk_u24 tk_seed; do timeout -k 10 90 ./$v 2048 $v 512 >> $GRAFT_REPO_ROOT/gpurun_out/r4_tk3.txt; done
