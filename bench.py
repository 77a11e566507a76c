#!/usr/bin/env python3
"""bench.py — device-resident guided_filter throughput (BASELINE.json metric).

Metric: GiB/s filtered (device-resident), guided_filter r=4, 2048^3 f32, 256^3 chunks
(BASELINE.json configs[2]; configs[1] is `--size 1024 --radius 2`). A step = one pass of the guided
filter over every 256^3 output chunk this rank owns (one fused-kernel launch on the HBM-resident
slab), inputs already resident when timing starts.

Multi-GPU (one process per GPU; `--gpus N` launches the N ranks itself through torch.distributed.run
when it is not already running under a launcher). The chunk work queue is split, as the reference's
chunk loop would be split (guided_filter.rs:260-316), into contiguous chunk rows along axis 0:
  * strong scaling (default): the one `size`^3 volume, rank g owns chunk rows [g*n/N, (g+1)*n/N)
    and holds them plus the 2r halo rows ArraySubsetOverlap would read (array_subset_overlap.rs:
    11-35), generated on its own device from the global synthetic definition;
  * weak scaling (`--scaling weak`): a (N*size, size, size) array, each rank owning a size^3 share.
No data-path collective: the process group carries the barrier and the max over ranks of the timed
region only. After timing, rank 0 checks a sample of its output chunks (corner, edge, interior)
against the oracle (oracle/, the reference's per-chunk algorithm) and reports `parity`.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

EPS = 2500.0
RADIUS = 4
N = 2048
CHUNK = 256
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); measured copy ~6.3 TB/s
ALGO_BYTES_PER_VOXEL = 8  # 4 B compulsory read + 4 B write
FLOAT_TOL = 1e-5  # |gpu - ref| <= 1e-5 * max(1, |ref|)
BASELINE_METRIC = "GiB/s filtered (device-resident), guided_filter r=4, 2048³ f32, 256³ chunks"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=N,
                    help="cube edge: the global volume (strong) or each rank's share (weak)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-chunks", type=int, default=0, help="chunks in the CPU sample")
    ap.add_argument("--parity-chunks", type=int, default=6,
                    help="output chunks checked against the oracle after timing (0: skip)")
    ap.add_argument("--share", default=None, metavar="G/N",
                    help="1-GPU proxy of one rank of an N-GPU strong split: run only rank G's "
                         "chunk rows (+ 2r halo) of the volume on this GPU (no process group)")
    ap.add_argument("--radius", type=int, default=RADIUS,
                    help="guided-filter radius (default 4 = the metric; 2 = config G2 at --size 1024)")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the other BASELINE configs timed after the headline (G2, the "
                         "config-T share, the config-P octant pyramid, the Gaussian)")
    ap.add_argument("--extra", default="g2,t_share,pyramid_octant,gaussian",
                    help="comma list of the extra legs to run")
    ap.add_argument("--dist-extra", default="t_series,p_pyramid",
                    help="with N > 1 ranks: the configs timed across the ranks after the headline "
                         "(configs[4]'s (t, z) blocks, configs[3]'s octant pyramid)")
    ap.add_argument("--dist-small", action="store_true",
                    help="the distributed legs on (32, 512^3) / 2048^3 instead of the BASELINE "
                         "sizes: rehearsing N ranks on one GPU (ZT_BENCH_ONE_DEVICE=1) only")
    ap.add_argument("--only-extra", default=None, metavar="LEG",
                    help="run only this extra leg, one untimed-warmup-free call (PMC passes: "
                         "tools/profile_pmc_legs.sh)")
    return ap.parse_args()


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def maybe_launch(args) -> None:
    """`--gpus N` outside a launcher: start the N ranks (torch.distributed.run, 127.0.0.1) as a
    child process before anything touches the GPU, and exit with its status."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if args.gpus != 1 and int(world_env) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
            sys.exit(2)
        return
    if args.gpus <= 1:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(subprocess.call(cmd, env=env))


def _affinity_count():
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None


def cpu_baseline(gshape, radius: int, nchunks: int = 0):
    """Reference algorithm (C restatement of guided_filter.rs, oracle/) on a bounded sample of
    the same workload: chunks of the same synthetic volume, 256^3 chunks, each with its 2r halo,
    every CPU of this process's affinity (rayon's default) capped at OMP_NUM_THREADS (the CPU
    share a GPU box grants), faithful incl. the dead 4th SAT. The default sample, 6
    chunks per thread, is about 15 s of CPU work at 0.4 GiB/s."""
    from oracle import oracle as O
    ncpu = os.cpu_count() or 1  # every CPU of the machine (nproc-like)
    try:  # the CPUs this process may run on (the GPU box grants a share of the machine)
        threads = max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        threads = ncpu
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:  # the share the box's scheduler grants (16 there)
        threads = min(threads, int(omp))
    nchunks = nchunks or 6 * threads
    grid = [-(-g // CHUNK) for g in gshape]
    coords = [((i * 3) % grid[0], (i * 5 + 1) % grid[1], (i * 7 + 2) % grid[2])
              for i in range(nchunks)]  # a diagonal walk through the grid (interior + edges)
    secs, vox = O.time_guided_filter_chunks(gshape, (CHUNK,) * 3, coords, EPS, radius, threads)
    gibs = vox * 4 / 2 ** 30 / secs
    # The reference's rayon pool would take every CPU of the affinity (guided_filter.rs:261-316).
    # A GPU box grants a share of its CPUs per GPU (OMP_NUM_THREADS), and worker pools stay within
    # it, so the full-affinity figure is extrapolated: one thread on 2 chunks gives the per-core
    # rate, the share run its parallel efficiency, and the estimate assumes that efficiency holds
    # up to every CPU of the affinity (memory-bounded like calculate_chunk_limit, not checked).
    full = None
    aff = _affinity_count() or ncpu
    if aff > threads:
        s1, v1 = O.time_guided_filter_chunks(gshape, (CHUNK,) * 3, coords[:2], EPS, radius, 1)
        g1 = v1 * 4 / 2 ** 30 / s1
        eff = min(1.0, gibs / (threads * g1))
        full = {"value": round(g1 * aff * eff, 4), "unit": "GiB/s", "cores": aff,
                "kind": "extrapolated", "per_core_gibs": round(g1, 5),
                "share_parallel_efficiency": round(eff, 3),
                "sample": f"1 thread on 2 chunks ({s1:.2f} s); estimate = per-core rate x "
                          f"{aff} CPUs x the {threads}-thread run's efficiency"}
    return {"value": round(gibs, 5), "unit": "GiB/s", "cores": threads, "kind": "port",
            "full_affinity": full,
            "host_cpus": ncpu, "affinity_cpus": _affinity_count(),
            "sample": f"{nchunks} chunks of 256^3 (r={radius}, 2r halo) of the same "
                      f"{'x'.join(map(str, gshape))} synthetic volume, {secs:.2f} s wall on "
                      f"{threads} threads (host: {ncpu} CPUs, {_affinity_count()} in this "
                      f"process's affinity, OMP_NUM_THREADS={omp or 'unset'}); "
                      f"C restatement of guided_filter.rs "
                      f"(oracle/zt_oracle.c, faithful incl. dead SAT)"}


def parity_sample(out_dev, a, gshape, radius: int, nchunks: int):
    """Compare a sample of this rank's output chunks (corner, edge, interior) with the oracle's
    per-chunk result (GuidedFilter::apply_chunk, guided_filter.rs:75-114), outside the timed
    region."""
    import numpy as np
    from oracle import oracle as O
    grid = [-(-g // CHUNK) for g in gshape]
    rows = range(a.out_z0 // CHUNK, -(-(a.out_z0 + a.out_nz) // CHUNK))
    coords = [c for c in O.sample_chunk_coords(grid, n_interior=max(1, nchunks - 4))
              if c[0] in rows]
    if not coords:
        coords = [(rows[0], 0, 0)]
    for c in O.sample_chunk_coords([len(rows)] + grid[1:]):
        cc = (rows[0] + c[0],) + tuple(c[1:])
        if len(coords) >= nchunks:
            break
        if cc not in coords:
            coords.append(cc)
    coords = coords[:max(nchunks, 1)]
    threads = max(1, min(16, os.cpu_count() or 1, len(coords)))
    t0 = time.perf_counter()
    refs = O.guided_filter_synth_chunks(gshape, (CHUNK,) * 3, coords, EPS, radius, threads)
    worst, exact, total = 0.0, 0, 0
    for (o0, osh, ref) in refs:
        z = o0[0] - a.out_z0
        got = out_dev[z:z + osh[0], o0[1]:o0[1] + osh[1], o0[2]:o0[2] + osh[2]].cpu().numpy()
        d = np.abs(got.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref.astype(np.float64)))
        worst = max(worst, float(d.max()))
        exact += int(np.count_nonzero(got == ref))
        total += got.size
    return {"max_rel": float(f"{worst:.3e}"), "tol": FLOAT_TOL, "ok": worst <= FLOAT_TOL,
            "chunks": [list(c) for c in coords], "bit_exact_frac": round(exact / total, 4),
            "oracle": "oracle/zt_oracle.c per-chunk apply_ndarray on the 2r-halo block",
            "secs": round(time.perf_counter() - t0, 2)}


def lib_hash() -> str:
    """sha256 of the shipped HIP library: the key a committed PMC traffic profile must match."""
    h = hashlib.sha256()
    with open(os.path.join(ROOT, "zarrs_tools_amd", "libzarrs_tools_amd.so"), "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def load_leg_traffic(leg: str):
    """Per-launch-set HBM traffic of an extra leg (profiles/pmc_traffic.json entries with
    "leg": name), only when measured on this exact library build; else None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        for e in d.get("entries", []):
            if e.get("leg") == leg and e.get("lib_sha256") == lib_hash():
                return e.get("hbm_bytes_per_call")
    except (OSError, ValueError, AttributeError):
        pass
    return None


def load_traffic(gshape, radius: int, world: int, share=None):
    """Per-launch HBM traffic from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json),
    only when it was measured on this exact library build and workload — the same global shape,
    radius and world size, and for a `--share G/N` proxy the same (G, N) share (entries without a
    "share" key describe the whole volume); else None."""
    e = load_traffic_entry(gshape, radius, world, share)
    return e.get("hbm_bytes_per_launch") if e else None


def load_sq(gshape, radius: int, world: int, share=None):
    """The SQ instruction counters per voxel (VALU, SALU, LDS, VMEM) and wave-cycle ratios of the
    same keyed PMC entry, or None."""
    e = load_traffic_entry(gshape, radius, world, share)
    if not e or "sq_per_voxel" not in e:
        return None
    return {"insts_per_voxel": e["sq_per_voxel"],
            "wave_cycle_ratios": e.get("sq_wave_cycle_ratios"),
            "source": "rocprofv3 --pmc SQ_* passes of the same build (tools/profile_pmc.sh)"}


def load_traffic_entry(gshape, radius: int, world: int, share=None):
    """The profiles/pmc_traffic.json entry of this build and workload (see load_traffic)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    want_share = list(share) if share is not None else None
    try:
        with open(path) as f:
            d = json.load(f)
        entries = d.get("entries", [d]) if isinstance(d, dict) else list(d)
        for e in entries:  # one entry per measured workload (G3 r=4, G2 r=2, ...)
            if (e.get("lib_sha256") == lib_hash() and list(e.get("global_shape", [])) == list(gshape)
                    and e.get("radius") == radius and e.get("world", 1) == world
                    and e.get("share") == want_share):
                return e
    except (OSError, ValueError, AttributeError):
        pass
    return None


# ---- the other BASELINE configs, timed after the headline on the same GPU -----------------------
# Each leg: HIP-event time on the launch stream (inputs resident), its roofline against the
# algorithmic bytes, the committed PMC traffic when keyed to this build, and a sampled parity
# check against the oracle (after timing). Never part of the headline `value`.

def _time_ms(fn, stream, warmup: int, reps: int) -> float:
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def _roof(algo_bytes: int, ms: float, traffic):
    gbs = algo_bytes / (ms / 1e3) / 1e9
    r = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes": int(algo_bytes),
         "traffic": traffic}
    if traffic:
        r["traffic_gbs"] = round(traffic / (ms / 1e3) / 1e9, 1)
    return r


def _max_rel(got, ref) -> float:
    import numpy as np
    d = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    return float((d / np.maximum(1.0, np.abs(ref.astype(np.float64)))).max())


def leg_g2(ctx, L, stream, warmup, reps):
    """configs[1]: guided_filter r=2 on 1024^3 f32, 256^3 chunks, one fused launch."""
    import torch
    import zarrs_tools_amd as zt
    from zarrs_tools_amd import _abi
    from zarrs_tools_amd.filter import _ptr
    size, radius = 1024, 2
    gshape = (size,) * 3
    a = zt.slab_assignment(0, 1, size, CHUNK, 2 * radius)
    dev = torch.device("cuda", torch.cuda.current_device())
    slab = torch.empty((a.in_nz, size, size), dtype=torch.float32, device=dev)
    out = torch.empty((a.out_nz, size, size), dtype=torch.float32, device=dev)
    _abi.check(L.zt_synth_step_noise_f32(ctx.handle, _ptr(slab), _abi.i64_array(slab.shape), 3,
                                         _abi.i64_array(gshape), a.in_z0, 0x5EED2025))
    gs, cs = _abi.i64_array(gshape), _abi.i64_array((CHUNK,) * 3)

    def step():
        _abi.check(L.zt_guided_filter_apply_slab(ctx.handle, 11, _ptr(slab), 11, _ptr(out), gs,
                                                 a.in_z0, a.in_nz, a.out_z0, a.out_nz, cs, EPS,
                                                 radius))
    ms = _time_ms(step, stream, warmup, reps)
    vox = size ** 3
    par = parity_sample(out, a, gshape, radius, 4)
    return {"config": "BASELINE configs[1]: guided_filter r=2 on 1024^3 f32, 256^3 chunks, "
                      "1 GPU device-resident", "ms": round(ms, 4),
            "value": round(vox * 4 / 2 ** 30 / (ms / 1e3), 3), "unit": "GiB/s",
            "roofline": dict(_roof(vox * ALGO_BYTES_PER_VOXEL, ms, load_traffic(gshape, radius, 1)),
                             sq=load_sq(gshape, radius, 1)),
            "parity": {k: par[k] for k in ("max_rel", "tol", "ok", "chunks", "bit_exact_frac")}}


def leg_t_share(ctx, L, stream, warmup, reps):
    """configs[4] per GPU: one rank's (t, z) block of the 8-GPU split of the (32, 1024^3) f32
    series in (4, 256^3) chunks (shard.block_split: 2 t-groups x 4 z-groups; an interior rank:
    16 output timepoints x 256 planes from 20 x 264 input planes), r=2, eps 2500, one
    GuidedFilter::apply_ndarray call on its halo'd box (the 4-D three-kernel path)."""
    import numpy as np
    import torch
    import zarrs_tools_amd as zt
    from zarrs_tools_amd import shard
    from zarrs_tools_amd.filter import ArraySubset
    from oracle import oracle as O
    gshape, chunk, world, radius = (32, 1024, 1024, 1024), (4, 256, 256, 256), 8, 2
    groups = shard.block_split(world, gshape, chunk, 2 * radius)
    rank = (groups[0] // 2) * groups[1] + groups[1] // 2
    a = shard.block_assignment(rank, world, gshape, chunk, 2 * radius, groups)
    x = zt.synth_box(a.in_start, a.in_shape, gshape, kind="float32", ctx=ctx)
    rel0 = tuple(o - i for o, i in zip(a.out_start, a.in_start))
    g = zt.GuidedFilter(EPS, radius)
    sub = ArraySubset(rel0, a.out_shape)
    res = {}

    def step():
        res["y"] = None  # the caching allocator hands the same block back
        res["y"] = g.apply_ndarray(x, sub, ctx=ctx)
    ms = _time_ms(step, stream, warmup, reps)
    y = res.pop("y")
    n = int(np.prod(a.out_shape))
    # parity: sampled (4, 32, 32, 32) output boxes (corner and interior of the share) against the
    # oracle's apply_ndarray on the box + its 2r halo from the global synthetic series (the
    # chunked result equals the whole-array one, tests/test_oracle.py)
    box = (4, 32, 32, 32)
    starts = [tuple(a.out_start), tuple(o + s // 2 for o, s in zip(a.out_start, a.out_shape)),
              tuple(o + s - b for o, s, b in zip(a.out_start, a.out_shape, box))]
    coords = [tuple(st // b for st, b in zip(s0, box)) for s0 in starts]
    worst = 0.0
    for (o0, osh, ref) in O.guided_filter_synth_chunks(gshape, box, coords, EPS, radius,
                                                       nthreads=len(coords)):
        sl = tuple(slice(p - q, p - q + s) for p, q, s in zip(o0, a.out_start, osh))
        worst = max(worst, _max_rel(y[sl].cpu().numpy(), ref))
    del x, y
    ctx.release_scratch()
    torch.cuda.empty_cache()
    return {"config": "BASELINE configs[4] per GPU: rank %d's (t, z) block of the 8-GPU split "
                      "of a (32, 1024^3) f32 series, (4, 256^3) chunks, r=2" % rank,
            "groups_t_z": list(groups), "output_box": [list(a.out_start), list(a.out_shape)],
            "input_box": [list(a.in_start), list(a.in_shape)], "ms": round(ms, 4),
            "value": round(n * 4 / 2 ** 30 / (ms / 1e3), 3), "unit": "GiB/s",
            "projected_8gpu_gibs": round(8 * n * 4 / 2 ** 30 / (ms / 1e3), 3),
            "roofline": _roof(n * ALGO_BYTES_PER_VOXEL, ms, load_leg_traffic("t_share")),
            "parity": {"max_rel": float(f"{worst:.3e}"), "tol": FLOAT_TOL,
                       "ok": worst <= FLOAT_TOL, "boxes": [list(c) for c in starts],
                       "box_shape": list(box)}}


def leg_pyramid_octant(ctx, L, stream, warmup, reps):
    """configs[3] per GPU: one rank's level-0 octant (2048^3 of the 4096^3 u16 volume) of the
    8-GPU zarrs_ome split, factor 2, 5 levels, the level-fused device pyramid."""
    import numpy as np
    import torch
    import zarrs_tools_amd as zt
    from oracle import oracle as O
    gshape, n, levels = (4096,) * 3, 2048, 5
    x = zt.synth_box((0, 0, 0), (n,) * 3, gshape, kind="uint16", ctx=ctx)
    res = {}

    def step():
        res["lv"] = None
        res["lv"] = zt.pyramid(x, (2, 2, 2), levels, ctx=ctx)
    ms = _time_ms(step, stream, warmup, reps)
    lv = res.pop("lv")
    nbytes = 2 * n ** 3 + sum(2 * int(np.prod(t.shape)) for t in lv)
    # parity (bit-exact): 64^3 level-0 blocks aligned to 2^5, their 5 levels from the oracle
    worst_ok = True
    starts = [(0, 0, 0), (n - 64,) * 3, (1024, 512, 1536)]
    for st in starts:
        cur = O.synth_block_nd(st, (64,) * 3, gshape, "uint16")
        for k, t in enumerate(lv):
            cur = O.downsample(cur, "uint16", (2, 2, 2), "uint16")
            f = 2 ** (k + 1)
            sl = tuple(slice(a // f, a // f + c) for a, c in zip(st, cur.shape))
            got = t[sl].cpu().numpy()
            worst_ok = worst_ok and np.array_equal(got, cur)
    del x, lv
    torch.cuda.empty_cache()
    return {"config": "BASELINE configs[3] per GPU: the level-0 octant 2048^3 of the 4096^3 "
                      "u16 volume, factor 2, 5 levels (zarrs_ome device pyramid)",
            "ms": round(ms, 4), "input_gvox_per_s": round(n ** 3 / (ms / 1e3) / 1e9, 3),
            "roofline": _roof(nbytes, ms, load_leg_traffic("pyramid_octant")),
            "parity": {"bit_exact": bool(worst_ok), "blocks": [list(s) for s in starts],
                       "block_shape": [64] * 3, "levels": levels}}


def leg_gaussian(ctx, L, stream, warmup, reps):
    """zarrs_filter gaussian sigma 1,1,1 half 3,3,3 on 1024^3 f32 (256^3 chunks)."""
    import numpy as np
    import torch
    import zarrs_tools_amd as zt
    from oracle import oracle as O
    n = 1024
    x = zt.synth_step_noise_f32((n,) * 3, ctx=ctx)
    y = torch.empty_like(x)
    g = zt.Gaussian([1.0] * 3, [3] * 3)
    a_in, a_out = zt.DeviceArray(x, (CHUNK,) * 3), zt.DeviceArray(y, (CHUNK,) * 3)
    ms = _time_ms(lambda: g.apply(a_in, a_out, ctx=ctx), stream, warmup, reps)
    # parity (bit-exact): 32^3 output boxes from the oracle on the box + its 3-voxel halo
    ok = True
    starts = [(0, 0, 0), (n - 32,) * 3, (500, 257, 640)]
    for st in starts:
        i0 = tuple(max(0, a - 3) for a in st)
        i1 = tuple(min(n, a + 32 + 3) for a in st)
        blk = O.synth_block_nd(i0, tuple(b - a for a, b in zip(i0, i1)), (n,) * 3, "float32")
        ref = O.gaussian_apply_ndarray(blk, [1.0] * 3, [3] * 3)
        sl = tuple(slice(a - b, a - b + 32) for a, b in zip(st, i0))
        got = y[tuple(slice(a, a + 32) for a in st)].cpu().numpy()
        ok = ok and np.array_equal(got, ref[sl])
    del x, y
    torch.cuda.empty_cache()
    return {"config": "gaussian sigma 1,1,1 half 3,3,3 on 1024^3 f32, 256^3 chunks (zarrs_filter "
                      "gaussian, SURVEY.md §8 (f)3)", "ms": round(ms, 4),
            "value": round(n ** 3 * 4 / 2 ** 30 / (ms / 1e3), 3), "unit": "GiB/s",
            "roofline": _roof(n ** 3 * 8, ms, load_leg_traffic("gaussian")),
            "parity": {"bit_exact": bool(ok), "boxes": [list(s) for s in starts],
                       "box_shape": [32] * 3}}


EXTRA_LEGS = {"g2": leg_g2, "t_share": leg_t_share, "pyramid_octant": leg_pyramid_octant,
              "gaussian": leg_gaussian}


def _dist_time(fn, dist, dev, one_dev, warmup: int, reps: int) -> float:
    """ms per rep of `fn` on this rank, between barriers, max over ranks."""
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize(dev)
    dist.barrier()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    tt = torch.tensor([ms], dtype=torch.float64, device="cpu" if one_dev else dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt[0])


def _dist_prepare(prepare, step, dist, dev, one_dev, warmup: int):
    """Allocate a distributed leg's inputs and run its untimed warm-up calls on every rank, then
    agree: an error on any rank (e.g. out of memory) makes every rank skip the leg together, so
    no rank is left waiting at a barrier the others never reach. Returns the error or None."""
    import torch
    err = None
    try:
        prepare()
        for _ in range(max(1, warmup)):
            step()
        torch.cuda.synchronize(dev)
    except Exception as e:
        err = f"{type(e).__name__}: {e}"
    if _dist_reduce([0.0 if err else 1.0], dist.ReduceOp.MIN, dist, dev, one_dev)[0] < 1.0:
        return err or "failed on another rank"
    return None


def _dist_reduce(vals, op, dist, dev, one_dev):
    import torch
    tt = torch.tensor(vals, dtype=torch.float64, device="cpu" if one_dev else dev)
    dist.all_reduce(tt, op=op)
    return [float(v) for v in tt]


def dist_t_series(ctx, rank, world, dist, dev, one_dev, warmup, reps, small=False):
    """configs[4] across the ranks: the (32, 1024^3) f32 series in (4, 256^3) chunks, r=2, split
    into the 8 (t, z) blocks of shard.block_split (2 t-groups x 4 z-groups); rank g runs blocks
    g, g + N, ... (one each at N = 8), each one GuidedFilter::apply_ndarray on its halo'd box
    (guided_filter.rs:240-319 per block of chunks). Time = max over ranks; every rank checks a
    (4, 32^3) output box of its first block against the oracle."""
    import numpy as np
    import zarrs_tools_amd as zt
    from zarrs_tools_amd import shard
    from zarrs_tools_amd.filter import ArraySubset
    from oracle import oracle as O
    gshape, chunk, nblk, radius = (32, 1024, 1024, 1024), (4, 256, 256, 256), 8, 2
    if small:  # --dist-small: the N-rank code path rehearsed on one GPU (never the reported size)
        gshape = (32, 512, 512, 512)
    groups = shard.block_split(nblk, gshape, chunk, 2 * radius)
    mine = [shard.block_assignment(b, nblk, gshape, chunk, 2 * radius, groups)
            for b in range(rank, nblk, world)]
    import torch
    subs = [ArraySubset(tuple(o - i for o, i in zip(a.out_start, a.in_start)), a.out_shape)
            for a in mine]
    g = zt.GuidedFilter(EPS, radius)
    res = {}

    def step():
        for x, sub in zip(res["x"], subs):
            res["y"] = None  # the caching allocator hands the same block back
            res["y"] = g.apply_ndarray(x, sub, ctx=ctx)
    err = _dist_prepare(lambda: res.update(x=[zt.synth_box(a.in_start, a.in_shape, gshape,
                                                           kind="float32", ctx=ctx)
                                              for a in mine]), step, dist, dev, one_dev, warmup)
    if err:
        res.clear()
        ctx.release_scratch()
        torch.cuda.empty_cache()
        return {"error": err}
    ms = _dist_time(step, dist, dev, one_dev, 0, reps)
    worst = float("inf")
    try:  # parity of the first block (recomputed after timing), local to the rank
        a = mine[0]
        y = g.apply_ndarray(res["x"][0], subs[0], ctx=ctx)
        box = (4, 32, 32, 32)
        s0 = tuple(o + s // 2 for o, s in zip(a.out_start, a.out_shape))
        coord = tuple(st // b for st, b in zip(s0, box))
        worst = 0.0
        for (o0, osh, ref) in O.guided_filter_synth_chunks(gshape, box, [coord], EPS, radius, 1):
            sl = tuple(slice(p - q, p - q + s) for p, q, s in zip(o0, a.out_start, osh))
            worst = max(worst, _max_rel(y[sl].cpu().numpy(), ref))
        del y
    except Exception:
        worst = float("inf")
    res.clear()
    ctx.release_scratch()
    torch.cuda.empty_cache()
    worst = _dist_reduce([worst], dist.ReduceOp.MAX, dist, dev, one_dev)[0]
    n = int(np.prod(gshape))
    return {"config": "BASELINE configs[4]: (32, 1024^3) f32 series, (4, 256^3) chunks, r=2, "
                      "its 8 (t, z) blocks over the ranks", "global_shape": list(gshape),
            "groups_t_z": list(groups),
            "blocks_per_rank": -(-nblk // world), "ms": round(ms, 4),
            "value": round(n * 4 / 2 ** 30 / (ms / 1e3), 3), "unit": "GiB/s",
            "scaling": "strong",
            "roofline_aggregate": _roof(n * ALGO_BYTES_PER_VOXEL, ms, None),
            "parity": {"max_rel_all_ranks": float(f"{worst:.3e}"), "tol": FLOAT_TOL,
                       "ok": worst <= FLOAT_TOL, "box_shape": list(box)}}


def dist_p_pyramid(ctx, rank, world, dist, dev, one_dev, warmup, reps, small=False):
    """configs[3] across the ranks: the 4096^3 u16 volume, factor 2, 5 levels, split into its 8
    level-0 octants (shard.octant_assignment, 2048^3 each: zarrs_ome --gpus 8); rank g runs
    octants g, g + N, ... (the level-fused device pyramid). Time = max over ranks; every rank
    checks its first octant's 5 levels bit-exactly on a 64^3 level-0 block."""
    import numpy as np
    import torch
    import zarrs_tools_amd as zt
    from zarrs_tools_amd import shard
    from oracle import oracle as O
    gshape, nblk, levels = (4096,) * 3, 8, 5
    if small:  # --dist-small (one-GPU rehearsal)
        gshape = (2048,) * 3
    mine = [shard.octant_assignment(b, nblk, gshape, (2, 2, 2), levels)
            for b in range(rank, nblk, world)]
    res = {}

    def step():
        for j, x in enumerate(res["x"]):
            res[j] = None
            res[j] = zt.pyramid(x, (2, 2, 2), levels, ctx=ctx)
    err = _dist_prepare(lambda: res.update(x=[zt.synth_box(a.start, a.shape, gshape,
                                                           kind="uint16", ctx=ctx)
                                              for a in mine]), step, dist, dev, one_dev, warmup)
    if err:
        res.clear()
        torch.cuda.empty_cache()
        return {"error": err}
    ms = _dist_time(step, dist, dev, one_dev, 0, reps)
    lv = res[0]
    nbytes = 2 * int(np.prod(gshape)) + nblk * sum(2 * int(np.prod(t.shape)) for t in lv)
    ok = False
    try:  # bit-exact levels of a 64^3 block of the first octant, local to the rank
        a = mine[0]
        st = tuple(s + n // 2 for s, n in zip(a.start, a.shape))  # 2^5-aligned
        cur = O.synth_block_nd(st, (64,) * 3, gshape, "uint16")
        ok = True
        for k, t in enumerate(lv):
            cur = O.downsample(cur, "uint16", (2, 2, 2), "uint16")
            f = 2 ** (k + 1)
            sl = tuple(slice((p - q) // f, (p - q) // f + c)
                       for p, q, c in zip(st, a.start, cur.shape))
            ok = ok and np.array_equal(t[sl].cpu().numpy(), cur)
    except Exception:
        ok = False
    del lv
    res.clear()
    torch.cuda.empty_cache()
    ok = _dist_reduce([1.0 if ok else 0.0], dist.ReduceOp.MIN, dist, dev, one_dev)[0] == 1.0
    return {"config": "BASELINE configs[3]: 4096^3 u16, factor 2, 5 levels (zarrs_ome device "
                      "pyramid), its 8 level-0 octants over the ranks", "global_shape": list(gshape),
            "octants_per_rank": -(-nblk // world), "ms": round(ms, 4),
            "input_gvox_per_s": round(int(np.prod(gshape)) / (ms / 1e3) / 1e9, 3),
            "scaling": "strong", "roofline_aggregate": _roof(nbytes, ms, None),
            "parity": {"bit_exact_all_ranks": bool(ok), "block_shape": [64] * 3,
                       "levels": levels}}


DIST_LEGS = {"t_series": dist_t_series, "p_pyramid": dist_p_pyramid}


def main():
    args = parse()
    maybe_launch(args)
    radius = args.radius
    import torch
    import torch.distributed as dist

    import zarrs_tools_amd as zt
    from zarrs_tools_amd import _abi
    from zarrs_tools_amd.filter import _ptr

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # ZT_BENCH_ONE_DEVICE=1 rehearses the N-rank path on a 1-GPU box: every rank on cuda:0, the
    # barrier / max-reduce over gloo (never used for a reported N>1 number)
    one_dev = os.environ.get("ZT_BENCH_ONE_DEVICE") == "1"
    if one_dev:
        local = 0
    # ZT_BENCH_DIST=1 under a launcher: join the process group even at one rank, so a 1-GPU box
    # runs the RCCL init / barrier / max-reduce of the N-GPU path (tests/test_bench_gpu.py)
    use_dist = world_env > 1 or ("WORLD_SIZE" in os.environ and
                                 os.environ.get("ZT_BENCH_DIST") == "1")
    backend = None
    if use_dist:
        torch.cuda.set_device(local)
        backend = "gloo" if one_dev else "nccl"
        if one_dev:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    world = dist.get_world_size() if use_dist else 1  # ranks RCCL actually joined
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    size = args.size
    gshape = (size * world, size, size) if args.scaling == "weak" else (size, size, size)
    share = None
    if args.share:  # (G, N): rank G's slab of an N-way split, timed alone on this GPU
        share = tuple(int(v) for v in args.share.split("/"))
        if world != 1 or args.scaling != "strong" or not 0 <= share[0] < share[1]:
            raise SystemExit("--share G/N: one process, strong scaling, 0 <= G < N")
        a = zt.slab_assignment(share[0], share[1], gshape[0], CHUNK, 2 * radius)
    else:
        a = zt.slab_assignment(rank, world, gshape[0], CHUNK, 2 * radius)
    stream = torch.cuda.current_stream(dev)
    ctx = zt.Context(local, stream)
    if args.only_extra:  # one call of one extra leg (its PMC passes); no headline
        L = _abi.lib()
        r = EXTRA_LEGS[args.only_extra](ctx, L, stream, 0, 1)
        print(json.dumps({"leg": args.only_extra, **r}), flush=True)
        ctx.close()
        return

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
                                                 radius))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if use_dist:
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
    if use_dist:
        dist.barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # HIP events on the launch stream
    if use_dist:
        tt = torch.tensor([wall, kern_ms], dtype=torch.float64,
                          device="cpu" if one_dev else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, kern_ms = float(tt[0]), float(tt[1])

    voxels_rank = a.out_nz * size * size  # rank 0's share (the largest, or equal)
    voxels_all = gshape[0] * size * size if share is None else voxels_rank
    ms_per_step = wall * 1000.0 / args.steps
    value = voxels_all * 4 / 2 ** 30 / (ms_per_step / 1000.0)
    achieved = voxels_rank * ALGO_BYTES_PER_VOXEL / (kern_ms / 1000.0) / 1e9  # GB/s per GPU
    traffic = load_traffic(gshape, radius, world, share)

    headline = share is None and ((size == N and radius == 4 and args.scaling == "strong") or (
        world == 1 and size == N and radius == 4))
    res = {
        "metric": BASELINE_METRIC if headline else
        f"GiB/s filtered (device-resident), guided_filter r={radius}, {size}³ f32, "
        f"{CHUNK}³ chunks",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": 1 if one_dev else world,
        "ranks": world,
        "dist_backend": backend,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SURVEY.md §8(d) step+noise, splitmix64 seed 0x5EED2025), generated "
                "on device",
        "config": {"workload": f"guided_filter eps={EPS:g} r={radius} on a "
                               f"{'x'.join(map(str, gshape))} f32 array, {CHUNK}^3 chunks, "
                               f"device-resident; rank g owns a z-slab of chunk rows + 2r halo",
                   "chunks_total": (gshape[0] // CHUNK) * (size // CHUNK) ** 2,
                   "chunks_rank0": (a.out_nz // CHUNK) * (size // CHUNK) ** 2,
                   "parallelism": f"chunk-rows x{world} ({args.scaling})"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_launch": voxels_rank * ALGO_BYTES_PER_VOXEL},
    }
    if traffic is not None:
        # the HBM bytes the kernel actually moves (PMC), per second of its launch: how close the
        # access pattern runs to the memory system's rate, next to the algorithmic `achieved`
        res["roofline"]["traffic_gbs"] = round(traffic / (kern_ms / 1000.0) / 1e9, 1)
        res["roofline"]["traffic_frac"] = round(res["roofline"]["traffic_gbs"] / HBM_PEAK_GBS, 4)
    res["roofline"]["sq"] = load_sq(gshape, radius, world, share)
    if share is not None:
        res["metric"] += f", rank {share[0]}'s share of a {share[1]}-GPU split (1-GPU proxy)"
        res["config"]["parallelism"] = f"share {share[0]}/{share[1]} on one GPU"
        res["share"] = {"rank": share[0], "world": share[1], "out_z": [a.out_z0, a.out_z0 + a.out_nz],
                        "in_z": [a.in_z0, a.in_z0 + a.in_nz],
                        # what N such GPUs would aggregate if every share ran this fast
                        "projected_aggregate_gibs": round(value * share[1], 3)}
    if rank == 0 and world == 1 and share is None and not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(gshape, radius, args.cpu_chunks)
        except Exception as e:  # the baseline is reported, never required
            res["cpu_baseline"] = {"value": None, "error": str(e)}
    if rank == 0 and args.parity_chunks > 0:
        res["parity"] = parity_sample(out, a, gshape, radius, args.parity_chunks)
        res["parity_max_rel"] = res["parity"]["max_rel"]
    if world == 1 and share is None and not args.no_extra and headline:
        del slab, out
        torch.cuda.empty_cache()
        extra = {}
        for name in [n for n in args.extra.split(",") if n]:
            try:
                t0 = time.perf_counter()
                extra[name] = EXTRA_LEGS[name](ctx, L, stream, 1, max(3, min(args.steps, 10)))
                extra[name]["wall_s"] = round(time.perf_counter() - t0, 2)
            except Exception as e:  # reported, never fatal to the headline line
                extra[name] = {"error": f"{type(e).__name__}: {e}"}
        res["extra_configs"] = extra
    if use_dist and world > 1 and share is None and not args.no_extra and headline:
        # configs[3] and [4] across the ranks (their own 8-way splits, round-robin over N ranks)
        del slab, out
        torch.cuda.empty_cache()
        dextra = {}
        for name in [n for n in args.dist_extra.split(",") if n]:
            t0 = time.perf_counter()
            dextra[name] = DIST_LEGS[name](ctx, rank, world, dist, dev, one_dev, 1, 3,
                                           small=args.dist_small)
            dextra[name]["wall_s"] = round(time.perf_counter() - t0, 2)
        res["dist_configs"] = dextra
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
