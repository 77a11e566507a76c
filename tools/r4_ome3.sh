#!/bin/bash
# zarrs_ome 2048^3 u16 end to end with per-phase wall clock (device path, store loop, 2 / 4 octant
# processes on the one GPU). GPU box, repo root.
set -e
timeout -k 10 900 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 4 > gpurun_out/r4_ome3_e2e.json 2> gpurun_out/r4_ome3_e2e.err
