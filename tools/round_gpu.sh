#!/bin/bash
# Full GPU round trip on the box: parity tests -> bench (with CPU baseline) -> rocprof trace +
# PMC HBM passes. Each step has its own time limit; any failure ends the script.
# Usage (from the repo root on the GPU box): tools/round_gpu.sh OUTDIR
set -u
OUT=${1:-gpurun_out/round}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed rc=$?"; tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
bash tools/profile_round.sh "$OUT/prof"
