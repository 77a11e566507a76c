#!/bin/bash
# rocprofv3 counter passes of the Gaussian LDS-DMA march (tools/bench_ops.py --only gaussian,
# 1024^3 sigma 1), each counter set in its own run. GPU box, repo root.
set -u
OUT=gpurun_out/r4_gauss_pmc
ROOT=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d "$ROOT/$OUT/$name" -o run --output-format csv -- \
    python3 "$ROOT/tools/bench_ops.py" --only gaussian --reps 1 > "$ROOT/$OUT/$name.log" 2>&1
  echo "$name rc=$?"
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
cd $ROOT
python3 tools/pmc_summary.py $OUT gauss_zyx $((1024*1024*1024)) 2 > $OUT/summary.txt
