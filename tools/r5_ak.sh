#!/bin/bash
# Round 5, call AK: the headline bench line of the final library, three times on one box
# (box-to-box spread comes from repeating the call).
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5ak
mkdir -p $O
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_$i.json 2> $O/bench_$i.err || exit 1; done
