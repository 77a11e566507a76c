#!/bin/bash
# rocprofv3 kernel trace of the ablation tool (per-kernel durations). Usage: tools/prof_ablate.sh OUT N
OUT=$1; N=${2:-2048}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/trace" -o run --output-format csv -- "$ROOT/tools/ablate" "$N" > "$ROOT/$OUT/ablate.log" 2>&1
echo "rc=$?"
