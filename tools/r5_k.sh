#!/bin/bash
# Round 5, call K: counters of the t-march form on config T's share geometry
# (tools/timetshare.hip): fabric bytes, L2 hits, SQ issue/wait. Each pass its own run.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in mz12 b8v2; do
  B=$GRAFT_REPO_ROOT/tools/exp/ts_$v
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${v}_fetch -o run -- $B 1024 $v > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${v}_write -o run -- $B 1024 $v > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/${v}_tcc -o run -- $B 1024 $v > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/${v}_sq1 -o run -- $B 1024 $v > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM --output-format csv -d $O/${v}_sq2 -o run -- $B 1024 $v > /dev/null 2>&1 || exit 1
done
echo done > $O/done
