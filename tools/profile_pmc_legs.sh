#!/bin/bash
# rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py's extra legs (one call each:
# bench.py --only-extra LEG), each counter in its own run (kernel-trace only). GPU box, repo root.
# Usage: tools/profile_pmc_legs.sh OUTDIR [legs...]
set -u
OUT=$1; shift
LEGS=${@:-g2 t_share pyramid_octant gaussian}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for leg in $LEGS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d "$ROOT/$OUT/${leg}_$c" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --only-extra $leg > "$ROOT/$OUT/${leg}_$c.log" 2>&1
    echo "$leg $c rc=$?"
  done
done
