#!/bin/bash
# round 3, GPU call 5: new GPU tests (CLI / zarrs_ome --gpus / casts / chunk limit, bench
# launcher + share proxy, the config-T real share), fused pyramid timing, ops rows, 8-way share proxies
set -u
OUT=gpurun_out/r3g5
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_cli_gpu.py tests/test_store_gpu.py tests/test_bench_gpu.py "tests/test_fullsize_gpu.py::test_t_share_4d_sampled_chunks" > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "FAIL|Error|max rel" $OUT/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_pyramid.py --size 4096 > $OUT/pyr4096.json 2>&1 || { echo pyr failed; tail $OUT/pyr4096.json; exit 1; }
cat $OUT/pyr4096.json
ZT_PYRAMID_UNFUSED=1 timeout -k 10 300 python -u tools/bench_pyramid.py --size 4096 > $OUT/pyr4096_unfused.json 2>&1 || exit 1
cat $OUT/pyr4096_unfused.json
for g in 0 3 7; do
  timeout -k 10 200 python -u bench.py --share $g/8 --steps 5 --warmup 2 --parity-chunks 2 --no-cpu-baseline > $OUT/share_${g}_8.json 2>&1 || exit 1
  tail -1 $OUT/share_${g}_8.json | cut -c1-300
done
timeout -k 10 600 python -u tools/bench_ops.py --reps 3 > $OUT/ops.jsonl 2> $OUT/ops.err || { tail $OUT/ops.err; exit 1; }
cut -c1-400 $OUT/ops.jsonl
