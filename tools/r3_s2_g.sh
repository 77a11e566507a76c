#!/bin/bash
# round 3 session 2, GPU call 8: integer stage 1 for u16 inputs (product header) vs the f64
# stage 1 (tools/gf_v4.hpp copy of the previous product), r=4 2048^3 and r=2 1024^3; f32 base
set -u
OUT=gpurun_out/r3s2g
mkdir -p $OUT
for v in u16old u16new u16old u16new base; do timeout -k 10 120 tools/tk_$v 2048 $v 512 >> $OUT/tk.txt 2>&1 || { cat $OUT/tk.txt; exit 1; }; done
for v in u16r2old u16r2new u16r2old u16r2new; do timeout -k 10 120 tools/tk_$v 1024 $v 1024 >> $OUT/tk.txt 2>&1 || { cat $OUT/tk.txt; exit 1; }; done
cat $OUT/tk.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_guided_filter_gpu.py tests/test_fullsize_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/pytest.log | head; exit 1; }
