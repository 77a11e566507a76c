#!/bin/bash
# Build (here, on the CPU host) tools/timek variants: tools/timek.sh build NAME "-DFLAGS"...
# Run (GPU box): tools/timek.sh run N NAME... — each under its own time limit.
set -u
cd "$(dirname "$0")"
if [ "$1" = build ]; then
  shift
  while [ $# -ge 2 ]; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize -Xclang -target-feature -Xclang -load-store-opt -I../zarrs_tools_amd/csrc $2 -o tk_$1 timek.hip 2>&1 | grep -v "not a recognized feature"
    shift 2
  done
else
  shift; n=$1; shift
  for v in "$@"; do timeout -k 10 120 ./tk_${v%%:*} $n $v ${v#*:} || exit 1; done
fi
