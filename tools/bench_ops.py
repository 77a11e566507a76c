#!/usr/bin/env python3
"""Device-resident rates of the other rows on the path: the zarrs_ome mean
pyramid (config P per GPU: a 2048^3 uint16 octant, factor 2, 5 levels) and the Gaussian
(zarrs_filter gaussian 1.0,1.0,1.0 3,3,3 on 1024^3 f32, docs/zarrs_filter.md:107). One JSON line
per operation with its HBM roofline fraction and a CPU baseline (the oracle's C restatement,
one thread, on a bounded sample of the same workload).

Algorithmic bytes: pyramid = level 0 read once + every level written once (2 B per u16
element; the fused launches never read an intermediate level back); Gaussian = 4 B read + 4 B written per voxel (the separable passes' intermediates are
not credited).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0


def timed(fn, stream, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def bench_pyramid(n, reps, levels, discrete=False, dtype="uint16"):
    import numpy as np
    import torch
    import zarrs_tools_amd as zt
    from oracle import oracle as O
    ctx = zt.default_context(0)
    x = zt.synth_u16((n, n, n))
    if dtype in ("uint8", "int8"):  # the low byte of the u16 noise: 256 values
        tt = torch.uint8 if dtype == "uint8" else torch.int8
        x = (x.view(torch.int16) & 0xFF).to(tt) if not discrete else \
            (x.view(torch.int16) & 0x7).to(tt)
    elif discrete:  # few distinct values, so the mode is not mostly a tie of eight
        x = (x.view(torch.int16) & 0x7).view(torch.uint16)
    esz = x.element_size()
    torch.cuda.synchronize()
    shapes = zt.pyramid_level_shapes((n, n, n), (2, 2, 2), levels)
    ms = timed(lambda: zt.pyramid(x, (2, 2, 2), levels, discrete=discrete, ctx=ctx),
               torch.cuda.current_stream(), reps)
    # parity (bit-exact): a 64^3 level-0 block aligned to 2^levels, its levels from the oracle
    lv = zt.pyramid(x, (2, 2, 2), levels, discrete=discrete, ctx=ctx)
    blk = x[:64, 64:128, 128:192].cpu().numpy()
    cur, exact = blk, True
    for k, t in enumerate(lv):
        cur = O.downsample(cur, dtype, (2, 2, 2), dtype, discrete=discrete)
        f = 2 ** (k + 1)
        got = t[:64 // f, 64 // f:128 // f, 128 // f:192 // f].cpu().numpy()
        exact = exact and np.array_equal(got, cur)
    del lv
    # compulsory bytes: level 0 read once + every level written once (fused launches never
    # read an intermediate level back); per_level: each level's input read + output written
    prev, nbytes, per_level = (n, n, n), esz * n ** 3, 0
    for s in shapes:
        per_level += esz * (int(np.prod(prev)) + int(np.prod(s)))
        nbytes += esz * int(np.prod(s))
        prev = s
    gbs = nbytes / (ms / 1e3) / 1e9
    # CPU: the oracle's level-1 downsample of a 256^3 sample (single thread)
    sample = O.synth_u16((256, 256, 256))
    if discrete:
        sample = (sample & 0x7).astype(np.dtype(dtype))
    elif dtype in ("uint8", "int8"):
        sample = (sample & 0xFF).astype(np.uint8).view(np.dtype(dtype))
    t0 = time.perf_counter()
    O.downsample(sample, dtype, (2, 2, 2), dtype, discrete=discrete)
    cpu_s = time.perf_counter() - t0
    return {"op": f"zarrs_ome {'mode (--discrete)' if discrete else 'mean'} pyramid "
                  "(device-resident)", "config":
            {"level0": [n] * 3, "dtype": dtype, "factor": [2, 2, 2], "levels": len(shapes)},
            "parity_bit_exact": bool(exact),
            "ms": round(ms, 4), "input_gvox_per_s": round(n ** 3 / (ms / 1e3) / 1e9, 3),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes": nbytes, "per_level_bytes": per_level},
            "cpu_baseline": {"input_gvox_per_s": round(256 ** 3 / cpu_s / 1e9, 4), "cores": 1,
                             "kind": "port", "sample": f"level 1 of a 256^3 {dtype} block, "
                             "oracle downsample (C restatement of downsample.rs:72-120)"}}


def bench_gaussian(n, reps):
    import torch
    import zarrs_tools_amd as zt
    from oracle import oracle as O
    ctx = zt.default_context(0)
    x = zt.synth_step_noise_f32((n, n, n))
    y = torch.empty_like(x)
    g = zt.Gaussian([1.0] * 3, [3] * 3)
    a_in, a_out = zt.DeviceArray(x, (256,) * 3), zt.DeviceArray(y, (256,) * 3)
    ms = timed(lambda: g.apply(a_in, a_out, ctx=ctx), torch.cuda.current_stream(), reps)
    gbs = n ** 3 * 8 / (ms / 1e3) / 1e9
    sample = O.synth_step_noise_f32((128, 128, 128))
    t0 = time.perf_counter()
    O.gaussian_apply_ndarray(sample, [1.0] * 3, [3] * 3)
    cpu_s = time.perf_counter() - t0
    return {"op": "gaussian sigma 1,1,1 half 3,3,3 (device-resident)",
            "config": {"shape": [n] * 3, "dtype": "float32", "chunk": [256] * 3},
            "ms": round(ms, 4), "gib_per_s": round(n ** 3 * 4 / 2 ** 30 / (ms / 1e3), 3),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes": n ** 3 * 8},
            "cpu_baseline": {"gib_per_s": round(128 ** 3 * 4 / 2 ** 30 / cpu_s, 4), "cores": 1,
                             "kind": "port", "sample": "128^3 f32 block, oracle Gaussian (C "
                             "restatement of gaussian.rs:110-119 / kernel.rs:17-73)"}}


def bench_guided4d(shape, chunk, radius, reps):
    """Config T per GPU: a (T, Z, Y, X) f32 time-series share, chunks
    (4, 256, 256, 256), eps 2500. 4-D arrays take the separable per-axis path."""
    import numpy as np
    import torch
    import zarrs_tools_amd as zt
    from oracle import oracle as O
    ctx = zt.default_context(0)
    x = zt.synth_step_noise_f32(tuple(shape))
    y = torch.empty_like(x)
    g = zt.GuidedFilter(2500.0, radius)
    a_in, a_out = zt.DeviceArray(x, chunk), zt.DeviceArray(y, chunk)
    ms = timed(lambda: g.apply(a_in, a_out, ctx=ctx), torch.cuda.current_stream(), reps)
    n = int(np.prod(shape))
    gbs = n * 8 / (ms / 1e3) / 1e9
    sshape = (4, 64, 64, 64)
    sample = O.synth_step_noise_f32(sshape)
    t0 = time.perf_counter()
    O.guided_filter_apply(sample, (4, 32, 32, 32), 2500.0, radius, nthreads=1)
    cpu_s = time.perf_counter() - t0
    del x, y
    torch.cuda.empty_cache()
    return {"op": f"guided_filter r={radius} 4-D time-series (device-resident)",
            "config": {"shape": list(shape), "dtype": "float32", "chunk": list(chunk),
                       "eps": 2500.0},
            "ms": round(ms, 4), "gib_per_s": round(n * 4 / 2 ** 30 / (ms / 1e3), 3),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes": n * 8},
            "cpu_baseline": {"gib_per_s": round(int(np.prod(sshape)) * 4 / 2 ** 30 / cpu_s, 5),
                             "cores": 1, "kind": "port",
                             "sample": f"{list(sshape)} f32 block in (4,32,32,32) chunks, oracle "
                             "guided filter (C restatement of guided_filter.rs)"}}


def bench_t_share(reps, radius=2, groups=None, rank=None):
    """Config T's real per-GPU share: rank `rank` of an 8-GPU split of the
    (32, 1024^3) f32 series in (4, 256^3) chunks, timed alone on this GPU. The chunk grid is
    split in (t, z) blocks of whole chunks (shard.block_assignment; `groups` = (t groups, z groups),
    default the input-minimising 2 x 4: 16 output timepoints x 256 planes from a 20 x 264-plane
    input, 1.29x stage-1 work, where rows along t (8 x 1) read 12 timepoints for 4, 3x). The
    rank's halo'd input block is generated from the global synthetic definition and filtered in
    one GuidedFilter::apply_ndarray call on its output box (chunked == whole with the 2r halo,
    SURVEY.md §0.2). Algorithmic bytes: 8 per OUTPUT voxel (halo reads not credited)."""
    import numpy as np
    import torch
    import zarrs_tools_amd as zt
    from zarrs_tools_amd import shard
    from zarrs_tools_amd.filter import ArraySubset
    from oracle import oracle as O
    ctx = zt.default_context(0)
    gshape, chunk, world = (32, 1024, 1024, 1024), (4, 256, 256, 256), 8
    halo = 2 * radius
    groups = tuple(groups) if groups else shard.block_split(world, gshape, chunk, halo)
    if rank is None:  # an interior block (largest input)
        rank = (groups[0] // 2) * groups[1] + groups[1] // 2 if groups[1] > 1 else groups[0] // 2
    a = shard.block_assignment(rank, world, gshape, chunk, halo, groups)
    x = zt.synth_box(a.in_start, a.in_shape, gshape, kind="float32", ctx=ctx)
    rel0 = tuple(o - i for o, i in zip(a.out_start, a.in_start))
    g = zt.GuidedFilter(2500.0, radius)
    sub = ArraySubset(rel0, a.out_shape)
    res = {}

    def run():
        res["y"] = None  # drop the previous output first (the caching allocator reuses it)
        res["y"] = g.apply_ndarray(x, sub, ctx=ctx)

    ms = timed(run, torch.cuda.current_stream(), reps)
    y = res["y"]
    n = int(np.prod(a.out_shape))
    gbs = n * 8 / (ms / 1e3) / 1e9
    # parity: one interior chunk of the share against the oracle's per-chunk result
    cidx = tuple((o + s // 2) // c for o, s, c in zip(a.out_start, a.out_shape, chunk))
    (o0, osh, ref), = O.guided_filter_synth_chunks(gshape, chunk, [cidx], 2500.0, radius,
                                                   nthreads=16)
    sl = tuple(slice(p - q, p - q + s) for p, q, s in zip(o0, a.out_start, osh))
    got = y[sl].cpu().numpy()
    rel = float((np.abs(got.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref))).max())
    del x, y, res
    ctx.release_scratch()
    torch.cuda.empty_cache()
    return {"op": f"guided_filter r={radius} 4-D, config T per-GPU share (device-resident)",
            "config": {"global_shape": list(gshape), "chunk": list(chunk), "world": world,
                       "groups_t_z": list(groups), "rank": rank,
                       "output_box": [list(a.out_start), list(a.out_shape)],
                       "input_box": [list(a.in_start), list(a.in_shape)],
                       "dtype": "float32", "eps": 2500.0,
                       "path": "one apply_ndarray call on the halo'd (t, z) block: 4-D three-kernel form (box3_march_kernel, g4_tab_kernel, box3_final_kernel)"},
            "ms": round(ms, 4), "gib_per_s": round(n * 4 / 2 ** 30 / (ms / 1e3), 3),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes": n * 8},
            "parity_chunk": list(cidx), "parity_max_rel": rel}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pyramid-size", type=int, default=2048)
    ap.add_argument("--gaussian-size", type=int, default=1024)
    ap.add_argument("--levels", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--t-shape", type=int, nargs=4, default=[4, 1024, 1024, 1024])
    ap.add_argument("--only", default="pyramid,gaussian,tshare")
    ap.add_argument("--t-groups", type=int, nargs=2, default=None,
                    help="config T share: (t groups, z groups) of the 8-GPU split")
    ap.add_argument("--t-rank", type=int, default=None)
    a = ap.parse_args()
    only = set(a.only.split(","))
    if "tshare" in only:
        print(json.dumps(bench_t_share(a.reps, groups=a.t_groups, rank=a.t_rank)), flush=True)
    if "guided4d" in only:
        print(json.dumps(bench_guided4d(a.t_shape, (4, 256, 256, 256), 2, a.reps)), flush=True)
        if only == {"guided4d"}:
            return
    if "pyramid" in only:
        print(json.dumps(bench_pyramid(a.pyramid_size, a.reps, a.levels)), flush=True)
    if "pyramid_u8" in only:  # the u8 mean pyramid (16-byte rows per lane: 2 level-3 columns)
        print(json.dumps(bench_pyramid(a.pyramid_size, a.reps, a.levels, False, "uint8")),
              flush=True)
    if "pyramid_i8" in only:  # the i8 mean and mode pyramids (the packed-byte kernel)
        for disc in (False, True):
            print(json.dumps(bench_pyramid(a.pyramid_size, a.reps, a.levels, disc, "int8")),
                  flush=True)
    if "pyramid_discrete" in only:
        for dt in ("uint16", "uint8"):
            print(json.dumps(bench_pyramid(a.pyramid_size, a.reps, a.levels, True, dt)),
                  flush=True)
    if "gaussian" in only:
        print(json.dumps(bench_gaussian(a.gaussian_size, a.reps)), flush=True)


if __name__ == "__main__":
    main()
