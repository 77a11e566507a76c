#!/bin/bash
# round 3, GPU call 2: microbenchmarks, new GPU tests (zarrs_ome --gpus, casts, chunk limit,
# fused pyramid), pyramid timing at 2048^3 / 4096^3.
set -u
OUT=gpurun_out/r3g2
mkdir -p $OUT
timeout -k 10 120 tools/ub_rates > $OUT/ubench.txt 2>&1 || { echo ubench failed; exit 1; }
cat $OUT/ubench.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_downsample_gpu.py tests/test_cli_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log; grep -E "FAIL|Error" $OUT/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_pyramid.py --size 4096 > $OUT/pyr4096.json 2>&1 || { echo pyr failed; tail $OUT/pyr4096.json; exit 1; }
cat $OUT/pyr4096.json
ZT_PYRAMID_UNFUSED=1 timeout -k 10 300 python -u tools/bench_pyramid.py --size 4096 > $OUT/pyr4096_unfused.json 2>&1 || exit 1
cat $OUT/pyr4096_unfused.json
timeout -k 10 120 tools/tk_base 2048 base 512 > $OUT/tk.txt 2>&1 || exit 1
cat $OUT/tk.txt
