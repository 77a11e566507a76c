#!/bin/bash
# Round 5, call C: zarrs_ome --gpus split tests (incl. 1 KiB pieces), the downsample tests (incl.
# the fused mode pyramid), bench.py with the extra legs.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_downsample_gpu.py tests/test_cli_gpu.py -k "gpus_split or pyramid or downsample" > $O/r5_c_tests.txt 2>&1
timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 > $O/r5_c_bench.json 2> $O/r5_c_bench.err
