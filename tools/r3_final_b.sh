#!/bin/bash
# Round-3 profiling pass B (GPU box, repo root): config G2 (r=2, 1024^3) bench line and its PMC
# traffic entry; 1-GPU proxies of three ranks' shares of the 8-way strong split; the other rows
# (T share, pyramid, Gaussian) with kernel-trace stats; config P's 4096^3 pyramid.
# Usage: tools/r3_final_b.sh [traffic json to merge into]
set -u
OUT=gpurun_out/${2:-r3fb}
ROOT=$(pwd)
mkdir -p $OUT
timeout -k 10 300 python3 -u bench.py --size 1024 --radius 2 --steps 20 --warmup 3 > $OUT/bench_g2.json 2> $OUT/bench_g2.err || { tail $OUT/bench_g2.err; exit 1; }
tail -1 $OUT/bench_g2.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  n=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 200 rocprofv3 --pmc $c -d $ROOT/$OUT/pmc_g2/$n -o run --output-format csv -- python3 $ROOT/bench.py --size 1024 --radius 2 --steps 1 --warmup 0 --parity-chunks 0 --no-cpu-baseline > $ROOT/$OUT/pmc_g2_$n.log 2>&1 || exit 1
done
cd $ROOT
cp ${1:-profiles/pmc_traffic.json} $OUT/pmc_traffic.json 2>/dev/null
python3 tools/make_traffic_json.py $OUT/pmc_g2 $OUT/pmc_traffic.json 1024 2 || exit 1
for g in 0 3 7; do
  timeout -k 10 200 python3 -u bench.py --share $g/8 --steps 10 --warmup 2 --parity-chunks 2 --no-cpu-baseline > $OUT/share_${g}_8.json 2>&1 || exit 1
  tail -1 $OUT/share_${g}_8.json | cut -c1-200
done
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/ops -o run --output-format csv -- python3 $ROOT/tools/bench_ops.py --reps 3 > $ROOT/$OUT/ops.jsonl 2> $ROOT/$OUT/ops.err || { tail $ROOT/$OUT/ops.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/pyr -o run --output-format csv -- python3 $ROOT/tools/bench_pyramid.py --size 4096 > $ROOT/$OUT/pyr4096.json 2> $ROOT/$OUT/pyr4096.err || { tail $ROOT/$OUT/pyr4096.err; exit 1; }
cd $ROOT
cut -c1-300 $OUT/ops.jsonl; grep '^{' $OUT/pyr4096.json | cut -c1-300
