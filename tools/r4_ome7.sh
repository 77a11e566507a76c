#!/bin/bash
# Pieced reads in read_to_device too: store/zarrs_ome/chain GPU tests, then zarrs_ome 2048^3 end
# to end (device path, store loop, octants) with default pieces and with whole rows. GPU box.
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_store_gpu.py tests/test_cli_gpu.py > gpurun_out/r4_ome7_pytest.txt 2>&1
timeout -k 10 500 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 4 --cli > gpurun_out/r4_ome7_e2e.json 2> gpurun_out/r4_ome7_e2e.err
ZT_READ_PIECE_KB=0 timeout -k 10 500 python -u tools/bench_ome_e2e.py --size 2048 > gpurun_out/r4_ome7_e2e_rows.json 2>> gpurun_out/r4_ome7_e2e.err
