#!/bin/bash
# Round 5: store -> store rates on the final library (tools/bench_e2e.py): 1024^3 r=4, the
# 4096 x 1024^2 r=4 volume, and config T's shape (32, 512^3) r=2 (now the t-march path).
set -u
OUT=gpurun_out/e2e5
mkdir -p $OUT
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 300 python3 tools/bench_e2e.py --size 1024 --radius 4 --cpu-chunks 32 > $OUT/bytes_r4.json 2> $OUT/bytes_r4.err || exit 1
timeout -k 10 400 python3 tools/bench_e2e.py --size 1024 --nz 4096 --radius 4 --repeat 1 > $OUT/bytes_r4_long.json 2> $OUT/bytes_r4_long.err || exit 1
timeout -k 10 600 python3 tools/bench_e2e.py --t 32 --size 512 --radius 2 --repeat 1 --cpu-chunks 16 > $OUT/t32_r2.json 2> $OUT/t32_r2.err || exit 1
