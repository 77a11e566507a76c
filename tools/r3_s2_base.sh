#!/bin/bash
# round 3 session 2, GPU call 1: whole GPU suite on the rebuilt library, then the default bench line
set -u
OUT=gpurun_out/r3s2a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "^FAILED|Error" $OUT/pytest.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2>&1 || { tail $OUT/bench.json; exit 1; }
tail -1 $OUT/bench.json
for pad in 0 32 64 128 0; do timeout -k 10 120 tools/tk_base 2048 pad$pad 512 $pad >> $OUT/tk_pad.txt 2>&1 || exit 1; done
cat $OUT/tk_pad.txt
timeout -k 10 300 tools/ablate 2048 > $OUT/ablate.txt 2>&1 || { cat $OUT/ablate.txt; exit 1; }
cat $OUT/ablate.txt
for v in base v4 v4ns base v4; do timeout -k 10 120 tools/tk_$v 2048 $v 512 >> $OUT/tk_v4.txt 2>&1 || exit 1; done
cat $OUT/tk_v4.txt
