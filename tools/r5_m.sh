#!/bin/bash
# Round 5, call M: mode pyramid with the sorting-network mode (tests + timings), then the whole GPU
# suite on the tree.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_downsample_gpu.py > $O/r5_m_ds_tests.txt 2>&1
timeout -k 10 300 python -u tools/bench_ops.py --only pyramid,pyramid_discrete --reps 5 > $O/r5_m_ops.jsonl 2> $O/r5_m_ops.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/r5_m_gpu_tests.txt 2>&1
