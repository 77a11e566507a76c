#!/bin/bash
# rocprofv3 counter passes of the config T per-GPU share (tools/bench_ops.py --only tshare: the
# three 4-D kernels on rank 5's (t, z) block of the (2, 4) split), each counter set in its own
# run (kernel-trace only, no sys/runtime trace). GPU box, repo root.
# Usage: tools/profile_pmc_tshare.sh OUTDIR
set -u
OUT=$1
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d "$ROOT/$OUT/$name" -o run --output-format csv -- \
    python3 "$ROOT/tools/bench_ops.py" --only tshare --reps 1 > "$ROOT/$OUT/$name.log" 2>&1
  echo "$name rc=$?"
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
cd "$ROOT"
V=$((16*256*1024*1024))
# bench_ops runs the share twice (one untimed call, then --reps 1): CALLS = 2
for k in box3_march g4_tab box3_final; do python3 tools/pmc_summary.py "$OUT" $k $V 2; done > "$OUT/summary.txt"
