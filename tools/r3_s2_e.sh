#!/bin/bash
# round 3 session 2, GPU call 5: wide-tile Gaussian variants; the product's wide-tile Gaussian:
# GPU tests, ops row with kernel trace
set -u
OUT=gpurun_out/r3s2e
ROOT=$(pwd)
mkdir -p $OUT
for v in base x256 x256t24 x256t24p2 x256t28 x192 x192t24p2 x128t64 base x256 x256t24 x256t24p2 x256t28 x192 x192t24p2 x128t64; do timeout -k 10 120 tools/tgs_$v 1024 $v >> $OUT/tgs.txt 2>&1 || { cat $OUT/tgs.txt; exit 1; }; done
cat $OUT/tgs.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gaussian_gpu.py tests/test_gaussian.py tests/test_bench_gpu.py::test_bench_rccl_process_group_at_one_rank > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/pytest.log | head; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/ops -o run --output-format csv -- python3 $ROOT/tools/bench_ops.py --reps 5 --only gaussian > $ROOT/$OUT/ops.jsonl 2> $ROOT/$OUT/ops.err || { tail $ROOT/$OUT/ops.err; exit 1; }
cd $ROOT
cut -c1-500 $OUT/ops.jsonl
grep gauss $OUT/ops/run_kernel_stats.csv | cut -c1-250
