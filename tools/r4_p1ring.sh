#!/bin/bash
# Fused kernel, stage-1 z-window ring at r <= 2: A/B timing (tools/timek.hip), then parity (the
# guided-filter GPU tests, full-size G2) and the G2 bench line. GPU box, repo root.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r4_p1ring
mkdir -p $O
cd tools/bin
for v in tk_r2base tk_r2ring tk_r2base tk_r2ring; do timeout -k 10 90 ./$v 1024 $v-1024 1024 >> $O/timek.txt || exit 1; done
for v in tk_r2base tk_r2ring; do timeout -k 10 90 ./$v 2048 $v-2048 1024 >> $O/timek.txt || exit 1; done
for v in tk_r2baseu16 tk_r2ringu16; do timeout -k 10 90 ./$v 1024 $v-1024 1024 >> $O/timek.txt || exit 1; done
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_guided_filter_gpu.py tests/test_fullsize_gpu.py tests/test_sharding_gpu.py > $O/tests.txt 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 300 python3 bench.py --size 1024 --radius 2 --no-cpu-baseline > $O/bench_g2.json 2> $O/bench_g2.err || exit 1
echo done
