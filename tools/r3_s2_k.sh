#!/bin/bash
# round 3 session 2: chunk-row grouping of the separable / four-kernel paths — guided GPU tests,
# the config-T share with kernel stats
set -u
OUT=gpurun_out/r3s2k
ROOT=$(pwd)
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_guided_filter_gpu.py tests/test_fullsize_gpu.py::test_t_share_4d_sampled_chunks > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/ops -o run --output-format csv -- python3 $ROOT/tools/bench_ops.py --reps 3 --only tshare > $ROOT/$OUT/ops.jsonl 2> $ROOT/$OUT/ops.err || { tail $ROOT/$OUT/ops.err; exit 1; }
cd $ROOT
cut -c1-300 $OUT/ops.jsonl
grep -E "g4_|box3|cast" $OUT/ops/run_kernel_stats.csv | cut -c1-200
