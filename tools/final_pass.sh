#!/bin/bash
# Final profiling pass of a round (GPU box, repo root), every step under its own time limit.
# Usage: tools/final_pass.sh [a|b|all]  (default all; a gpurun call is capped at 20 minutes, so the
# round-6 pass ran a and b as two calls)
#   a: bench.py line (headline + extra legs, cpu_baseline, parity); kernel-trace stats of it;
#      PMC passes of the headline kernel (SQ, FETCH, WRITE, TCC) and of G2; FETCH / WRITE of the
#      other extra legs; pmc_traffic.json keyed to this build; the bench line again with traffic
#   b: the GPU test suite, smoke(), and the N-rank bench path rehearsed on the one GPU (2 and 4
#      ranks, ZT_BENCH_ONE_DEVICE=1, --dist-small for the distributed legs)
set -u
PART=${1:-all}
OUT=gpurun_out/final
ROOT=$(pwd)
mkdir -p $OUT
if [ "$PART" = a ] || [ "$PART" = all ]; then
timeout -k 10 500 python3 bench.py > $OUT/bench_first.json 2> $OUT/bench_first.err || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/kt -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --parity-chunks 0 --steps 5 --warmup 1 > $ROOT/$OUT/kt.log 2>&1 ) || exit 1
tools/profile_pmc.sh $OUT/pmc --steps 1 --warmup 0 --parity-chunks 0 || exit 1
python3 tools/pmc_summary.py $OUT/pmc gf3d $((2048*2048*2048)) > $OUT/pmc_summary.txt
PASSES="sq1 sq2 fetch write" tools/profile_pmc.sh $OUT/pmc_g2 --size 1024 --radius 2 --steps 1 --warmup 0 --parity-chunks 0 || exit 1
python3 tools/pmc_summary.py $OUT/pmc_g2 gf3d $((1024*1024*1024)) > $OUT/pmc_g2_summary.txt
rm -f profiles/pmc_traffic.json
python3 tools/make_traffic_json.py $OUT/pmc profiles/pmc_traffic.json 2048 4 || exit 1
python3 tools/make_traffic_json.py $OUT/pmc_g2 profiles/pmc_traffic.json 1024 2 || exit 1
tools/profile_pmc_legs.sh $OUT/legs t_share pyramid_octant gaussian || exit 1
python3 tools/make_traffic_json.py --legs $OUT/legs profiles/pmc_traffic.json t_share pyramid_octant gaussian || exit 1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
timeout -k 10 500 python3 bench.py > $OUT/bench_final.json 2> $OUT/bench_final.err || exit 1
echo a-done > $OUT/done_a
fi
if [ "$PART" = b ] || [ "$PART" = all ]; then
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || exit 1
for n in 2 4; do
  ZT_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus $n --steps 3 --warmup 1 --no-cpu-baseline --parity-chunks 2 --dist-small > $OUT/rehearse_${n}ranks.json 2> $OUT/rehearse_${n}ranks.err || exit 1
done
echo b-done > $OUT/done_b
fi
