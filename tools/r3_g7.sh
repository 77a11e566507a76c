#!/bin/bash
# round 3, GPU call 7: A/B of the cleaned kernel, the whole GPU test suite, pyramid / shares / ops
set -u
OUT=gpurun_out/r3g7
mkdir -p $OUT
bash tools/r3_g6.sh > $OUT/ab.txt 2>&1 || { cat $OUT/ab.txt; exit 1; }
cat gpurun_out/r3g6/tk.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "^FAILED|Error" $OUT/pytest.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_pyramid.py --size 4096 > $OUT/pyr4096.json 2>&1 || exit 1
cat $OUT/pyr4096.json
ZT_PYRAMID_UNFUSED=1 timeout -k 10 200 python -u tools/bench_pyramid.py --size 4096 > $OUT/pyr4096_unfused.json 2>&1 || exit 1
cat $OUT/pyr4096_unfused.json
for g in 0 3 7; do
  timeout -k 10 200 python -u bench.py --share $g/8 --steps 5 --warmup 2 --parity-chunks 2 --no-cpu-baseline > $OUT/share_${g}_8.json 2>&1 || exit 1
  tail -1 $OUT/share_${g}_8.json | cut -c1-300
done
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2>&1 || exit 1
tail -1 $OUT/bench.json | cut -c1-600
