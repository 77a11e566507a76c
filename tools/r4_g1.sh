#!/bin/bash
# round 4: GPU tests of the changed paths, then config T share timings
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cli_gpu.py tests/test_downsample_gpu.py tests/test_store_gpu.py > gpurun_out/r4_g1_pytest.txt 2>&1
timeout -k 10 400 python -u tools/bench_ops.py --only tshare --reps 3 --t-groups 2 4 >> gpurun_out/r4_tshare.jsonl 2>> gpurun_out/r4_tshare.err
timeout -k 10 400 python -u tools/bench_ops.py --only tshare --reps 3 --t-groups 4 2 >> gpurun_out/r4_tshare.jsonl 2>> gpurun_out/r4_tshare.err
