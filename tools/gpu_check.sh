#!/bin/bash
# One GPU round trip: parity tests, then the bench (only if the tests did not crash).
OUT=${1:-gpurun_out}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > $OUT/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc
tail -3 $OUT/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1
  echo bench_rc=$?
  tail -1 $OUT/bench.log | cut -c1-400
fi
