#!/bin/bash
# Store -> store measurements of the round (GPU box, repo root), each with the CPU store -> store
# baseline on a sample of output chunks. Usage: tools/e2e_round.sh OUTNAME
set -u
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 300 python3 tools/bench_e2e.py --size 1024 --radius 2 --cpu-chunks 32 > $OUT/bytes_r2.json 2> $OUT/bytes_r2.err || exit 1
timeout -k 10 300 python3 tools/bench_e2e.py --size 1024 --radius 4 --cpu-chunks 32 > $OUT/bytes_r4.json 2> $OUT/bytes_r4.err || exit 1
timeout -k 10 400 python3 tools/bench_e2e.py --size 1024 --nz 4096 --radius 4 --repeat 1 > $OUT/bytes_r4_long.json 2> $OUT/bytes_r4_long.err || exit 1
timeout -k 10 300 python3 tools/bench_e2e.py --size 1024 --radius 2 --codec zstd --level 1 --repeat 1 --cpu-chunks 16 > $OUT/zstd_r2.json 2> $OUT/zstd_r2.err || exit 1
timeout -k 10 400 python3 tools/bench_e2e.py --t 16 --size 512 --radius 2 --repeat 1 --cpu-chunks 16 > $OUT/t16_r2.json 2> $OUT/t16_r2.err || exit 1
