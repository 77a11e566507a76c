#!/bin/bash
# Default torch-free octant workers (512 MiB read pieces): zarrs_ome GPU tests, 2048^3 u16 end to
# end in-process and as CLI processes. GPU box, repo root.
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cli_gpu.py -k "ome" > gpurun_out/r4_ome6_pytest.txt 2>&1
timeout -k 10 500 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 4 --cli > gpurun_out/r4_ome6_e2e.json 2> gpurun_out/r4_ome6_e2e.err
