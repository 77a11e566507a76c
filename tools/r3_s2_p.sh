#!/bin/bash
# round 3 session 2: smoke() as the driver runs it, then one short default bench line
set -u
OUT=gpurun_out/r3s2p
mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-700
