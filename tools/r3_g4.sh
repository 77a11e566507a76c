#!/bin/bash
# round 3, GPU call 4: CLI/zarrs_ome tests after the pending-metadata change, fused pyramid timing
set -u
OUT=gpurun_out/r3g4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cli_gpu.py tests/test_store_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "FAIL|Error" $OUT/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_pyramid.py --size 4096 > $OUT/pyr4096.json 2>&1 || { echo pyr failed; tail $OUT/pyr4096.json; exit 1; }
cat $OUT/pyr4096.json
ZT_PYRAMID_UNFUSED=1 timeout -k 10 300 python -u tools/bench_pyramid.py --size 4096 > $OUT/pyr4096_unfused.json 2>&1 || exit 1
cat $OUT/pyr4096_unfused.json
