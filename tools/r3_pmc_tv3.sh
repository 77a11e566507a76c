#!/bin/bash
# SQ counter passes of the v3 kernel and the round-2 kernel (tools/tv3_r4, 1024^3 r=4).
# Usage (GPU box, repo root): tools/r3_pmc_tv3.sh OUTDIR
set -u
OUT=$1
ROOT=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for w in 1 2; do
  timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/kt$w -o run --output-format csv -- $ROOT/tools/tv3_r4 1024 512 $w > $ROOT/$OUT/kt$w.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $ROOT/$OUT/sq1_$w -o run --output-format csv -- $ROOT/tools/tv3_r4 1024 512 $w > $ROOT/$OUT/sq1_$w.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM -d $ROOT/$OUT/sq2_$w -o run --output-format csv -- $ROOT/tools/tv3_r4 1024 512 $w > $ROOT/$OUT/sq2_$w.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_IFETCH SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_ANY -d $ROOT/$OUT/sq3_$w -o run --output-format csv -- $ROOT/tools/tv3_r4 1024 512 $w > $ROOT/$OUT/sq3_$w.log 2>&1 || echo "sq3 pass failed (counter names)"
done
cd $ROOT
for w in 1 2; do cat $OUT/kt$w.log | tail -2; done
find $OUT -name "*counter_collection.csv" | head
