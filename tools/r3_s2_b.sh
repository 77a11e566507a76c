#!/bin/bash
# round 3 session 2, GPU call 2: 2-WG-per-CU tile (64x16, 512 threads) A/B; ops rows (T share,
# Gaussian, pyramid) kernel stats; Gaussian PMC read/write bytes
set -u
OUT=gpurun_out/r3s2b
ROOT=$(pwd)
mkdir -p $OUT
for v in base t16 t16s base t16; do timeout -k 10 120 tools/tk_$v 2048 $v 512 >> $OUT/tk.txt 2>&1 || { cat $OUT/tk.txt; exit 1; }; done
cat $OUT/tk.txt
for v in base n512 t64 t64n1024 x128 t48 t48w4 t48n512 base n512 t48 t48w4; do timeout -k 10 120 tools/tgs_$v 1024 $v >> $OUT/tgs.txt 2>&1 || { cat $OUT/tgs.txt; exit 1; }; done
cat $OUT/tgs.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/ops -o run --output-format csv -- python3 $ROOT/tools/bench_ops.py --reps 3 > $ROOT/$OUT/ops.jsonl 2> $ROOT/$OUT/ops.err || { tail $ROOT/$OUT/ops.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c -d $ROOT/$OUT/g_$c -o run --output-format csv -- python3 $ROOT/tools/bench_ops.py --reps 1 --only gaussian > $ROOT/$OUT/g_$c.log 2>&1 || exit 1
done
cd $ROOT
cut -c1-600 $OUT/ops.jsonl
find $OUT/ops -name "*kernel_stats.csv" | xargs cat | cut -c1-250
