#!/bin/bash
# Round 5, call AH: Hx column swizzle (GF_HX_SWZ=1) against the product, r = 4 and r = 2
# (tools/timek.hip 2048^3), then the LDS bank-conflict counter of both r = 4 builds.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O/r5ah
( cd tools/exp && for v in s0 swz r2s0 r2swz s0 swz r2s0 r2swz s0 swz; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O/r5ah/times.txt || exit 1; done ) || exit 1
cd /tmp && export TMPDIR=/tmp
for v in s0 swz; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/r5ah/pmc_$v -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/exp/tk_$v 2048 $v 512 > $O/r5ah/pmc_$v.log 2>&1 || exit 1
done
