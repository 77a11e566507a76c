#!/bin/bash
# Round profile: kernel trace + stats of the default bench command, and PMC HBM-traffic passes
# (FETCH_SIZE and WRITE_SIZE in separate runs, kernel-trace only) at the bench's full size.
# Usage (on the GPU box, from the repo root): tools/profile_round.sh OUTDIR
set -u
OUT=$1
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/trace" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-extra > "$ROOT/$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$ROOT/$OUT/fetch" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-extra > "$ROOT/$OUT/fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$ROOT/$OUT/write" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-extra > "$ROOT/$OUT/write.log" 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
