#!/bin/bash
# Round-end check with the final library: the whole -m gpu suite, then the default bench line
# (which must now carry the PMC traffic keyed to this build). GPU box, repo root.
set -e
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_suite_tests.txt 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/r4_suite_bench.json 2> gpurun_out/r4_suite_bench.err
