#!/bin/bash
# Round-3 profiling pass A (GPU box, repo root): the whole GPU suite on this library, the default
# bench line, its kernel-trace stats, the PMC passes of the fused kernel (SQ, FETCH, WRITE, TCC)
# and the traffic entry keyed to this build. Each step under its own limit; any failure ends it.
set -u
OUT=gpurun_out/${1:-r3fa}
ROOT=$(pwd)
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $OUT/pytest.log | head; exit 1; }
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-300
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/kt -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --parity-chunks 0 --steps 5 --warmup 1 > $ROOT/$OUT/kt.log 2>&1 ) || exit 1
grep gf3d $OUT/kt/run_kernel_stats.csv | cut -c1-200
bash tools/profile_pmc.sh $OUT/pmc --steps 1 --warmup 0 --parity-chunks 0 || exit 1
python3 tools/pmc_summary.py $OUT/pmc gf3d $((2048*2048*2048)) > $OUT/pmc_summary.txt
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json 2>/dev/null
python3 tools/make_traffic_json.py $OUT/pmc $OUT/pmc_traffic.json 2048 4 || exit 1
cat $OUT/pmc_summary.txt
