#!/bin/bash
# Round 5, call AI: instruction-cache behaviour of the headline kernel unrolled by 18 steps (the
# two-step prefetch, tk_s0) against 9 (tk_p1): rocprofv3 --list-avail (SQC counters), then one
# --pmc pass of SQ_IFETCH / SQC_ICACHE_* per build when available.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5ai
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
C=""
for c in SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY; do grep -q "$c" $O/avail.txt && C="$C $c"; done
echo "counters:$C" > $O/counters.txt
[ -n "$C" ] || exit 0
for v in s0 p1; do
  timeout -s KILL 90 rocprofv3 --pmc $C -d $O/pmc_$v -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/exp/tk_$v 2048 $v 512 > $O/pmc_$v.log 2>&1 || exit 1
done
