#!/bin/bash
# rocprofv3 counter passes for the guided-filter kernel (run on the GPU box from the repo root).
# Usage: [PASSES="fetch write lds"] tools/profile_pmc.sh OUTDIR [bench args...]
# Each --pmc pass is its own run (kernel-trace only; no sys/runtime trace with counters).
set -u
OUT=$1; shift
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PASSES=${PASSES:-"sq1 sq2 fetch write tcc"}
run() {  # name counters...
  local name=$1; shift
  [[ " $PASSES " == *" $name "* ]] || return 0
  timeout -k 10 240 rocprofv3 --pmc "$@" -d "$ROOT/$OUT/$name" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-extra "${BENCH_ARGS[@]}" > "$ROOT/$OUT/$name.log" 2>&1
  echo "$name rc=$?"
}
BENCH_ARGS=("$@")
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
run lds SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU || exit 1
