#!/bin/bash
# The whole -m gpu suite on the final tree. GPU box, repo root.
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_suite2_tests.txt 2>&1
