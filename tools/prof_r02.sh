#!/bin/bash
# Round-2 profiling pass (GPU box, repo root): kernel-trace stats of one bench run, the PMC
# traffic + SQ counters of the fused kernel, and a 2-rank one-device rehearsal of bench --gpus 2.
set -u
OUT=gpurun_out/$1; shift
mkdir -p $OUT
ROOT=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/kt -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --parity-chunks 0 --steps 5 --warmup 1 > $ROOT/$OUT/kt.log 2>&1 ) || exit 1
tools/profile_pmc.sh $OUT/pmc --steps 1 --warmup 0 --parity-chunks 0 || exit 1
python3 tools/pmc_summary.py $OUT/pmc gf3d $((2048*2048*2048)) > $OUT/pmc_summary.txt
ZT_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --parity-chunks 2 > $OUT/rehearse2.json 2> $OUT/rehearse2.err || exit 1
