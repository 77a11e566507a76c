#!/bin/bash
# Round 5, call P: the GPU suite on the product library after the box3_final F32 fix (the
# re-reading form of the march took v = 0 for radii whose ring does not fit in registers).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/r5_p_tests.txt 2>&1
