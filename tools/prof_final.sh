#!/bin/bash
# Round-end profiling pass (GPU box, repo root): bench.py line (with cpu_baseline and parity),
# kernel-trace stats of the bench, PMC counter passes of the fused kernel (SQ, FETCH, WRITE,
# TCC), the traffic JSON keyed to this build, and the other rows (bench_ops) with their kernel
# stats. Usage: tools/prof_final.sh OUTNAME
set -u
OUT=gpurun_out/$1
mkdir -p $OUT
ROOT=$(pwd)
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/kt -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --parity-chunks 0 --steps 5 --warmup 1 > $ROOT/$OUT/kt.log 2>&1 ) || exit 1
tools/profile_pmc.sh $OUT/pmc --steps 1 --warmup 0 --parity-chunks 0 || exit 1
python3 tools/pmc_summary.py $OUT/pmc gf3d $((2048*2048*2048)) > $OUT/pmc_summary.txt
python3 tools/make_traffic_json.py $OUT/pmc $OUT/pmc_traffic.json 2048 4 || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/ops -o run --output-format csv -- python3 $ROOT/tools/bench_ops.py --reps 3 > $ROOT/$OUT/ops.jsonl 2> $ROOT/$OUT/ops.err ) || exit 1
