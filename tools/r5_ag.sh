#!/bin/bash
# Round 5, call AG: the GPU suite and smoke() on the final tree.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/r5ag_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r5ag_smoke.txt 2>&1
