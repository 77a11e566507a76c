#!/bin/bash
# Round 5, call AL: the N-rank bench path rehearsed on one GPU (ZT_BENCH_ONE_DEVICE=1: every rank
# on cuda:0, gloo barrier / max-reduce), 2 and 4 ranks, final library.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5al
mkdir -p $O
export ZT_BENCH_ONE_DEVICE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 3 --warmup 1 --no-extra --no-cpu-baseline > $O/bench_n$n.json 2> $O/bench_n$n.err || exit 1
done
