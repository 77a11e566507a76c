#!/bin/bash
# zarrs_ome --gpus N with pre-spawned octant workers: the zarrs_ome GPU tests, then the 2048^3 u16
# end-to-end (device path, store loop, 2 and 4 octant processes on the one GPU). GPU box, repo root.
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cli_gpu.py -k "ome" > gpurun_out/r4_ome2_pytest.txt 2>&1
timeout -k 10 900 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 4 > gpurun_out/r4_ome2_e2e.json 2> gpurun_out/r4_ome2_e2e.err
