#!/bin/bash
# zarrs_ome --gpus N with torch-free octant workers (hiprt.py) against torch workers
# (ZT_OCTANT_TORCH=1) and with non-coherent pinned buffers (ZT_PINNED_FLAGS): the zarrs_ome GPU
# tests, then the 2048^3 u16 end to end. GPU box, repo root.
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cli_gpu.py -k "ome" > gpurun_out/r4_ome5_pytest.txt 2>&1
timeout -k 10 500 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 4 --cli > gpurun_out/r4_ome5_e2e.json 2> gpurun_out/r4_ome5_e2e.err
ZT_OCTANT_TORCH=1 timeout -k 10 500 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 4 > gpurun_out/r4_ome5_e2e_torch.json 2>> gpurun_out/r4_ome5_e2e.err
ZT_PINNED_FLAGS=0x80000000 timeout -k 10 500 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 4 > gpurun_out/r4_ome5_e2e_nc.json 2>> gpurun_out/r4_ome5_e2e.err
ZT_READ_PIECE_KB=524288 timeout -k 10 500 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 4 > gpurun_out/r4_ome5_e2e_pieces.json 2>> gpurun_out/r4_ome5_e2e.err
ZT_READ_PIECE_KB=32 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cli_gpu.py -k "gpus_split" > gpurun_out/r4_ome5_pieces_pytest.txt 2>&1
