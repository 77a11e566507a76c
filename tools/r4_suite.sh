#!/bin/bash
# Round-end check with the final library: the whole -m gpu suite, the default bench line (which
# must carry the PMC traffic keyed to this build), and zarrs_ome end to end incl. fresh CLI
# processes. GPU box, repo root.
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_suite_tests.txt 2>&1
timeout -k 10 240 python3 bench.py > gpurun_out/r4_suite_bench.json 2> gpurun_out/r4_suite_bench.err
timeout -k 10 400 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 4 --cli > gpurun_out/r4_suite_ome.json 2> gpurun_out/r4_suite_ome.err
