#!/bin/bash
# round 4: zarrs_ome end to end (fused device pyramid + pipelined ingest) and its kernel trace
set -e
timeout -k 10 900 python -u tools/bench_ome_e2e.py --size 2048 --gpus 2 > gpurun_out/r4_ome_e2e.json 2> gpurun_out/r4_ome_e2e.err
W=/tmp/zt_ome_prof && mkdir -p $W
timeout -k 10 300 python -u -c "
from zarrs_tools_amd import store as S
S.create_array('$W/in.zarr', 'uint16', (1024,)*3, (256,)*3)
S.write_synth('$W/in.zarr', S.SYNTH_U16, nthreads=16)
"
cd /tmp && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4_ome_prof -o run -- python3 -m zarrs_tools_amd.zarrs_ome $W/in.zarr $W/out.zarr > $GRAFT_REPO_ROOT/gpurun_out/r4_ome_prof.log 2>&1
