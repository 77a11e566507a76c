#!/usr/bin/env python3
"""bench.py — device-resident guided_filter throughput (BASELINE.json metric).

Metric: GiB/s filtered (device-resident), guided_filter r=4, 2048^3 f32, 256^3 chunks.
A step = one pass of the guided filter over every 256^3 chunk of this rank's 2048^3 f32 volume
(one fused-kernel launch on the HBM-resident array), inputs already resident when timing starts.

Multi-GPU (torchrun, one rank per GPU): weak scaling. The global array is (N*2048, 2048, 2048);
rank g owns the chunk rows of z in [g*2048, (g+1)*2048) and holds them plus the 2r halo rows the
reference's per-chunk ArraySubsetOverlap would read, generated on its own device from the global
synthetic definition. No data-path collective: the process group is used only for the barrier
and the max-over-ranks of the timed region.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

EPS = 2500.0
RADIUS = 4
N = 2048
CHUNK = 256
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); measured copy ~6.29 TB/s
ALGO_BYTES_PER_VOXEL = 8  # 4 B compulsory read + 4 B write


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=N, help="per-rank cube edge (default 2048)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-chunks", type=int, default=0, help="chunks in the CPU sample")
    ap.add_argument("--radius", type=int, default=RADIUS,
                    help="guided-filter radius (default 4 = the metric; 2 = config G2 at --size 1024)")
    return ap.parse_args()


def cpu_baseline(size: int, nchunks: int = 0):
    """Reference algorithm (C restatement of guided_filter.rs, oracle/) on a bounded sample of
    the same workload: chunks of the same 2048^3 synthetic volume, r=4, 256^3 chunks, each with
    its 2r halo, all host threads (rayon default), faithful incl. the dead 4th SAT. The default
    sample, 6 chunks per thread (6 GiB of output), is about 15 s of CPU work at 0.4 GiB/s."""
    from oracle import oracle as O
    ncpu = os.cpu_count() or 1
    threads = max(1, min(16, ncpu))  # the GPU box grants a 16-CPU share
    nchunks = nchunks or 6 * threads
    coords = []
    g = size // CHUNK
    for i in range(nchunks):  # a diagonal walk through the chunk grid (interior + edge chunks)
        coords.append(((i * 3) % g, (i * 5 + 1) % g, (i * 7 + 2) % g))
    secs, vox = O.time_guided_filter_chunks((size,) * 3, (CHUNK,) * 3, coords, EPS, RADIUS,
                                            threads)
    gibs = vox * 4 / 2 ** 30 / secs
    return {"value": round(gibs, 5), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{nchunks} chunks of 256^3 (r={RADIUS} halo) of the same {size}^3 synthetic "
                      f"volume, {secs:.2f} s wall on {threads} threads; C restatement of "
                      f"guided_filter.rs (oracle/zt_oracle.c, faithful incl. dead SAT)"}


def load_traffic(size: int):
    """Per-launch HBM traffic from the committed rocprofv3 PMC summary, if one matches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("size") == size and d.get("radius") == RADIUS:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    global RADIUS
    args = parse()
    RADIUS = args.radius
    import torch
    import torch.distributed as dist

    import zarrs_tools_amd as zt
    from zarrs_tools_amd import _abi
    from zarrs_tools_amd.filter import _ptr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    size = args.size
    gshape = (size * world, size, size)
    a = zt.slab_assignment(rank, world, gshape[0], size, 2 * RADIUS)
    stream = torch.cuda.current_stream(dev)
    ctx = zt.Context(local, stream)

    slab = torch.empty((a.in_nz, size, size), dtype=torch.float32, device=dev)
    out = torch.empty((a.out_nz, size, size), dtype=torch.float32, device=dev)
    L = _abi.lib()
    _abi.check(L.zt_synth_step_noise_f32(ctx.handle, _ptr(slab), _abi.i64_array(slab.shape), 3,
                                         _abi.i64_array(gshape), a.in_z0, 0x5EED2025))
    torch.cuda.synchronize(dev)

    gs = _abi.i64_array(gshape)
    cs = _abi.i64_array((CHUNK,) * 3)

    def step():
        _abi.check(L.zt_guided_filter_apply_slab(ctx.handle, 11, _ptr(slab), 11, _ptr(out), gs,
                                                 a.in_z0, a.in_nz, a.out_z0, a.out_nz, cs, EPS,
                                                 RADIUS))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # HIP events on the launch stream
    if world > 1:
        tt = torch.tensor([wall, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, kern_ms = float(tt[0]), float(tt[1])

    voxels_rank = a.out_nz * size * size
    voxels_all = voxels_rank * world
    ms_per_step = wall * 1000.0 / args.steps
    value = voxels_all * 4 / 2 ** 30 / (ms_per_step / 1000.0)
    achieved = voxels_rank * ALGO_BYTES_PER_VOXEL / (kern_ms / 1000.0) / 1e9  # GB/s per GPU
    traffic = load_traffic(size)

    res = {
        "metric": f"GiB/s filtered (device-resident), guided_filter r={RADIUS}, {size}^3 f32, "
                  f"{CHUNK}^3 chunks",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SURVEY.md §8(d) step+noise, splitmix64 seed 0x5EED2025), generated "
                "on device",
        "config": {"workload": f"guided_filter eps={EPS:g} r={RADIUS} on {size}^3 f32 per GPU, "
                               f"{CHUNK}^3 chunks, device-resident (global array "
                               f"{gshape[0]}x{size}x{size}, z-slab per rank + 2r halo)",
                   "chunks_per_gpu": (size // CHUNK) ** 3, "parallelism": f"chunk-rows x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_launch": voxels_rank * ALGO_BYTES_PER_VOXEL},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(size, args.cpu_chunks)
        except Exception as e:  # the baseline is reported, never required
            res["cpu_baseline"] = {"value": None, "error": str(e)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
