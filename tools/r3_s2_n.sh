#!/bin/bash
# round 3 session 2: SQ counter passes of the fused Gaussian (bench_ops --only gaussian, 1024^3)
set -u
OUT=gpurun_out/r3s2n
ROOT=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" -d $ROOT/$OUT/$name -o run --output-format csv -- python3 $ROOT/tools/bench_ops.py --reps 1 --only gaussian > $ROOT/$OUT/$name.log 2>&1 || exit 1; }
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM
run tcc TCC_HIT_sum TCC_MISS_sum
cd $ROOT
python3 tools/pmc_summary.py $OUT gauss_zyx $((1024*1024*1024*2)) > $OUT/summary.txt
cat $OUT/summary.txt
