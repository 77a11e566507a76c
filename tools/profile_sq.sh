#!/bin/bash
# SQ counter passes (instruction mix, waits, LDS activity) for the fused kernel on the bench's
# default workload; each --pmc pass is its own run (kernel-trace only). Usage: OUTDIR [bench args]
set -u
OUT=$1; shift
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d "$ROOT/$OUT/$name" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-extra --steps 1 --warmup 0 "${BENCH_ARGS[@]}" > "$ROOT/$OUT/$name.log" 2>&1
  echo "$name rc=$?"
}
BENCH_ARGS=("$@")
run a SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA || exit 1
run b SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_CYCLES SQ_WAVES || exit 1
run c SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH || exit 1
run d SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_IFETCH SQ_BUSY_CYCLES || exit 1
