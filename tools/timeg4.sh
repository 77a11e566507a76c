#!/bin/bash
# Build (CPU host) tools/timeg4 variants: tools/timeg4.sh build NAME "-DFLAGS"...
# Run (GPU box): tools/timeg4.sh run N NAME... — each under its own time limit.
set -u
cd "$(dirname "$0")"
if [ "$1" = build ]; then
  shift
  while [ $# -ge 2 ]; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize $2 -o tg_$1 timeg4.hip ../zarrs_tools_amd/csrc/cast.hip 2>&1 | grep -v "not a recognized"
    shift 2
  done
else
  shift; n=$1; shift
  for v in "$@"; do timeout -k 10 120 ./tg_$v $n $v || exit 1; done
fi
