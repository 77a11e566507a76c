#!/usr/bin/env python3
"""Config P (BASELINE.json configs[3]): the zarrs_ome 2x mean pyramid, 5 levels, of a 4096^3
uint16 volume, device-resident, one process per GPU with octant ownership (SURVEY.md §8(e),
zarrs_tools_amd.shard.octant_assignment): rank g generates its level-0 box of the global
synthetic volume on its device (zt_synth_box) and computes levels 1-5 of it (zt_pyramid_downsample)
with no exchange; levels whose chunks span boxes are assembled on the host only when written to
a store (not part of this device-resident measurement).

    python tools/bench_pyramid.py [--gpus N] [--size 4096] [--levels 5] [--steps K] [--warmup W]

--gpus N outside a launcher starts the N ranks itself (torch.distributed.run, 127.0.0.1). With
--size 4096 at N = 1 the single GPU holds the whole 32 GiB volume. Prints one JSON line: input
Gvox/s over all ranks, the max-over-ranks time per pyramid, the per-GPU algorithmic HBM rate
(level 0 read once + every level written once) and its roofline fraction, and a bit-exact
check of one 64^3 block of each level against the oracle (rank 0, outside the timed region)."""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--levels", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1",
               f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    import numpy as np
    import torch
    import torch.distributed as dist
    import zarrs_tools_amd as zt
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    one_dev = os.environ.get("ZT_BENCH_ONE_DEVICE") == "1"  # rehearsal: all ranks on cuda:0
    if one_dev:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if one_dev:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    shape, factor = (a.size,) * 3, (2, 2, 2)
    asg = zt.octant_assignment(rank, world, shape, factor, a.levels)
    ctx = zt.default_context(local)
    box = zt.synth_box(asg.start, asg.shape, shape, "uint16", ctx=ctx)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()

    def step():
        return zt.pyramid(box, factor, asg.local_levels, ctx=ctx)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    levels = None
    for _ in range(a.steps):
        levels = None  # free the previous step's levels first (caching allocator reuse)
        levels = step()
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = (time.perf_counter() - t0) / a.steps
    kern = e0.elapsed_time(e1) / a.steps / 1e3
    if world > 1:
        t = torch.tensor([wall, kern], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, kern = float(t[0]), float(t[1])
    # compulsory bytes (the roofline basis): level 0 read once + every level written once (the
    # fused launches never read an intermediate level back); per_level_bytes: each level's
    # input read + output written, as one launch per level moves them
    prev, per_level = asg.shape, 0
    nbytes = 2 * int(np.prod(asg.shape))
    for lv in levels:
        per_level += 2 * (int(np.prod(prev)) + int(np.prod(lv.shape)))
        nbytes += 2 * int(np.prod(lv.shape))
        prev = tuple(lv.shape)
    res = None
    if rank == 0:
        from oracle import oracle as O
        # bit-exact sample: level k's first 32^3 block from the oracle's downsample of the same
        # input block of level k-1 (level 0 = the synthetic volume)
        ok, src = True, None
        for k, lv in enumerate(levels):
            n = min(32, lv.shape[0])
            inp = (O.synth_block_nd(asg.start, (2 * n,) * 3, shape, "uint16") if k == 0
                   else levels[k - 1][:2 * n, :2 * n, :2 * n].cpu().numpy())
            want = O.downsample(inp, "uint16", factor, "uint16")
            ok = ok and bool(np.array_equal(lv[:n, :n, :n].cpu().numpy(), want))
        gbs = nbytes / kern / 1e9
        res = {"op": "zarrs_ome 2x mean pyramid, octant-owned (device-resident)",
               "config": {"level0": list(shape), "dtype": "uint16", "factor": list(factor),
                          "levels": asg.local_levels, "rank0_box": list(asg.shape),
                          "grid": list(asg.grid)},
               "n_gpus": 1 if one_dev else world, "ranks": world, "steps": a.steps,
               "ms_per_pyramid": round(wall * 1e3, 4),
               "input_gvox_per_s": round(np.prod(shape) / wall / 1e9, 2),
               "roofline_rank0": {"bound": "hbm", "achieved": round(gbs, 1),
                                  "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(gbs / HBM_PEAK_GBS, 4),
                                  "kernel_ms": round(kern * 1e3, 4),
                                  "algorithmic_bytes": nbytes,
                                  "per_level_bytes": per_level},
               "parity": {"bit_exact_sample": ok, "oracle": "oracle downsample of 64^3 blocks"}}
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
