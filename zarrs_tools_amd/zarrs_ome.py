"""``zarrs_ome`` for the accelerated path: an OME-Zarr (v0.5) multiscale group from a Zarr V3
array, every level computed by the HIP downsample kernel over the store.

    python -m zarrs_tools_amd.zarrs_ome INPUT OUTPUT [FACTOR,...] [--max-levels N] [--discrete]
        [--gaussian-sigma S,...] [--gaussian-kernel-half-size H,...] [--physical-size P,...]
        [--physical-units U,...] [--name NAME] [--group-attributes JSON]
        [--exists erase|exit|overwrite] [--ome-zarr-version 0.5] [reencoding args]
        [--device D] [--chunk-limit N]

Follows src/bin/zarrs_ome.rs (0.7.2):
* the output group gets --group-attributes (:317-323); --exists erase / exit / overwrite (:326-339);
* level 0 is a copy of the input, or with any reencoding argument (ZarrReencodingArgs,
  lib.rs:274-377) the input reencoded into the new encoding (:341-366);
* array 0's attributes move to the group, without "_zarrs" (:368-377);
* level i is the downsample of level i-1 (:515-738): read back from the output store as the
  reference does, or — when level 0 and its pyramid fit 80 % of the free device memory
  (`--no-device-resident` turns it off) — computed from the previous level kept in HBM, level 0
  read once and every level written once (the same kernels, so the same bits). Its encoding is the
  input's with zarrs_ome's per-level shapes (:528-560): a sharded input gets the shard shape
  min(shard, output) and the inner chunk min(inner chunk, output); otherwise the chunk shape
  min(chunk, output), which get_array_builder_reencode applies only to sharded outputs
  (lib.rs:623-646), so an unsharded level keeps the input's chunk grid. The loop stops when every
  axis has factor 1 or extent 1 (:731-737);
* each level adds a dataset with the cumulative f32 scale of input/output shape ratios and
  translation (scale - 1) / 2 (:570-578, :716-726);
* axes are named by the array's dimension names, else by index, typed by --physical-units (space,
  time, "channel", or a custom unit, :379-446); --physical-size is the multiscale's
  coordinateTransformations (:448-452); the multiscales "type" is "mode", "average" or "gaussian"
  (:468-475).
Mean downsampling, the mode with --discrete (ties by the smallest value: the documented deviation,
DESIGN.md §2), or with --gaussian-sigma a Gaussian of each level's input before the mean
(apply_chunk_continuous_gaussian, :236-271; kernel half size default ceil(3 sigma), :494-502;
ignored with --discrete, :638-646).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import shutil
import sys
import tempfile
import time

import numpy as np

from . import _abi
from . import store as S
from .zarrs_filter import (REENCODE_KEYS, _add_reencode_args, _device_ok, allocation_refused,
                           encoding_of, read_to_device, write_from_device)

VERSION = "zarrs_tools_amd 0.2 (MI355X)"

# OME-NGFF 0.5 units (ome_zarr_metadata 0.2.3 AxisUnit: Space | Time | Custom)
SPACE_UNITS = {
    "angstrom", "attometer", "centimeter", "decimeter", "exameter", "femtometer", "foot",
    "gigameter", "hectometer", "inch", "kilometer", "megameter", "meter", "micrometer", "mile",
    "millimeter", "nanometer", "parsec", "petameter", "picometer", "terameter", "yard",
    "yoctometer", "yottameter", "zeptometer", "zettameter"}
TIME_UNITS = {
    "attosecond", "centisecond", "day", "decisecond", "exasecond", "femtosecond", "gigasecond",
    "hectosecond", "hour", "kilosecond", "megasecond", "microsecond", "millisecond", "minute",
    "nanosecond", "petasecond", "picosecond", "second", "terasecond", "yoctosecond",
    "yottasecond", "zeptosecond", "zettasecond"}


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="zarrs_ome")
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("factor", nargs="?", default=None,
                    type=lambda s: [int(x) for x in s.split(",")])
    ap.add_argument("--ome-zarr-version", default="0.5", choices=["0.5"])
    ap.add_argument("--max-levels", type=int, default=10)
    ap.add_argument("--physical-size", default=None,
                    type=lambda s: [float(x) for x in s.split(",")])
    ap.add_argument("--physical-units", default=None, type=lambda s: s.split(","))
    ap.add_argument("--discrete", action="store_true")
    ap.add_argument("--gaussian-sigma", default=None,
                    type=lambda s: [float(x) for x in s.split(",")])
    ap.add_argument("--gaussian-kernel-half-size", default=None,
                    type=lambda s: [int(x) for x in s.split(",")])
    ap.add_argument("--name", default=None)
    ap.add_argument("--group-attributes", default=None)
    ap.add_argument("--exists", choices=["erase", "exit", "overwrite"], default="erase")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--gpus", type=int, default=1,
                    help="one process per GPU: octant-owned levels (mean / mode), or every "
                         "level split by output chunk rows (--gaussian-sigma)")
    ap.add_argument("--gpu-devices", default=None, type=lambda s: [int(v) for v in s.split(",")],
                    help="with --gpus N: process g runs on device LIST[g] (default 0..N-1; "
                         "e.g. 0,0 rehearses a 2-GPU run on one device)")
    ap.add_argument("--no-device-resident", action="store_true",
                    help="read every level back from the store (the reference's loop)")
    _add_reencode_args(ap)  # adds --chunk-limit too
    return ap


def level_scale(scale, in_shape, out_shape):
    """relative_scale *= (input / output) as f32 per axis (zarrs_ome.rs:570-578)."""
    f32 = np.float32
    return [float(f32(f32(s) * f32(int(i) // int(o)))) for s, i, o in
            zip(scale, in_shape, out_shape)]


def level_translation(scale):
    """(s - 1.0) * 0.5 in f32 (zarrs_ome.rs:721-723)."""
    f32 = np.float32
    return [float(f32(f32(f32(s) - f32(1.0)) * f32(0.5))) for s in scale]


def level_encoding(info: "S.ArrayInfo", out_shape) -> dict:
    """zarrs_ome.rs:528-560: the per-level chunk (and shard) shape of level i from level i-1."""
    if info.chunk_shape != info.inner_chunk_shape:  # sharded input
        return {"shard_shape": [min(c, s) for c, s in zip(info.chunk_shape, out_shape)],
                "chunk_shape": [min(g, s) for g, s in zip(info.inner_chunk_shape, out_shape)]}
    return {"chunk_shape": [min(c, s) for c, s in zip(info.chunk_shape, out_shape)]}


def axis_of(name: str, unit):
    """units_to_axis (zarrs_ome.rs:390-432)."""
    if unit is None:
        return {"name": name}
    if unit in SPACE_UNITS:
        return {"name": name, "type": "space", "unit": unit}
    if unit in TIME_UNITS:
        return {"name": name, "type": "time", "unit": unit}
    if unit == "channel":
        return {"name": name, "type": "channel"}
    return {"name": name, "unit": unit}


PENDING = S.PENDING_METADATA  # metadata of a level not finished yet (host/zt_zarr.hpp)
_hold_metadata = S.hold_metadata
_publish_metadata = S.publish_metadata


def _reencode_level0(src, dst, encoding, nthreads, log, device: int = 0):
    """Reencode::apply for level 0 (zarrs_ome.rs:341-366, reencode.rs:128-223): the input's data
    in the new encoding, chunk row by chunk row; with --data-type every element is converted on
    the device with the reference's `as` (zt_reencode_cast, reencode.rs:58-77)."""
    info = S.open_array(src)
    dt_out = encoding.get("data_type") or info.data_type
    if dt_out not in S.NUMPY:
        raise _abi.UnsupportedDataType(_abi.ERR_UNSUPPORTED_DATA_TYPE,
                                       f"unsupported data type {dt_out}")
    convert = dt_out != info.data_type
    if convert and not _device_ok(device):
        raise _abi.FilterError(_abi.ERR_DEVICE, "zarrs_ome --data-type: no HIP device")
    S.create_output_like(src, dst, dt_out, encoding)
    _hold_metadata(dst)
    out = S.open_array(dst)
    cz = out.chunk_shape[0]
    ctx = None
    for z0 in range(0, info.shape[0], cz):
        n = min(cz, info.shape[0] - z0)
        block = S.read_array(src, [z0] + [0] * (info.ndim - 1), [n] + list(info.shape[1:]),
                             nthreads=nthreads)
        if convert:
            import torch
            from . import filter as F
            ctx = ctx or F.default_context(device)
            x = torch.from_numpy(block).to(torch.device("cuda", device))
            if info.data_type == "bfloat16":
                x = x.view(torch.bfloat16)
            y = F.reencode_cast(x, dt_out, ctx)
            if dt_out == "bfloat16":
                y = y.view(torch.uint16)
            block = y.cpu().numpy()
        S.write_array(dst, block, [z0] + [0] * (info.ndim - 1), nthreads=nthreads)
    _publish_metadata(dst)
    log(f"0: reencode {src} -> {dst} ({out.data_type} {list(out.shape)})")


def _ingest(path, device: int, nthreads: int, log):
    """Level 0 into HBM (pipelined decode || H2D); (None, False) when an allocation is refused
    (the store path then runs the levels)."""
    t1 = time.perf_counter()
    try:
        x = read_to_device(path, device, nthreads)
    except RuntimeError as e:
        if not allocation_refused(e):
            raise  # storage / codec errors are real failures
        return None, False
    log(f"   level 0 -> device in {time.perf_counter() - t1:.2f}s")
    return x, True


def _device_pyramid_fits(info, gauss, device: int, frac: float = 0.8, sharing: int = 1,
                         host_share: int = 1) -> bool:
    """Level 0 + the pyramid (< 1/7 of level 0 for 2x factors, bounded by level 0 here) + the
    f32 Gaussian of the largest level, against `frac` of the free device memory (split between
    `sharing` processes on one device), and level 0's pinned host copy against `frac` of the
    available host memory (split `host_share` ways)."""
    import torch
    n = int(np.prod(info.shape))
    esz = S.NUMPY[info.data_type]().itemsize
    need = 2 * n * esz + (4 * n if gauss is not None else 0)
    free, _ = torch.cuda.mem_get_info(device)
    return (need <= frac * free / max(sharing, 1)
            and n * esz <= frac * S.host_available_bytes() / max(host_share, 1))


def _box_chunks(bstart, bshape, chunk, shape):
    """Chunk-grid index ranges of the chunks a box touches, and its chunk-aligned inner box
    [i0, i1) (whole chunks inside the box; a chunk cut by the array end counts as whole)."""
    lo = [b // c for b, c in zip(bstart, chunk)]
    hi = [-(-(b + n) // c) for b, n, c in zip(bstart, bshape, chunk)]
    i0 = [-(-b // c) * c for b, c in zip(bstart, chunk)]
    i1 = [(b + n) if b + n == s else (b + n) // c * c
          for b, n, c, s in zip(bstart, bshape, chunk, shape)]
    return lo, hi, i0, i1


def _box_levels_no_torch(lvl0: str, info0, assign, factor, discrete: bool, device: int,
                         nthreads: int):
    """The device part of an octant worker without torch (ZT_NO_TORCH=1, hiprt.py): the box of
    level 0 streamed into HBM chunk row by chunk row (a host thread decodes row k+1 into one of
    three pinned buffers while row k is copied on a stream, as read_to_device does), levels 1..L
    by zt_pyramid_downsample (per-level zt_downsample_apply_ndarray past the fused levels, as
    F.pyramid's callers do), and every level copied back to pinned host memory.
    Returns (levels as numpy arrays, read seconds, kernel seconds, buffers to keep alive, phase
    seconds)."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    from . import filter as F
    from . import hiprt as H
    from .zarrs_filter import _read_pieces
    t0 = time.perf_counter()
    H.set_device(device)
    dt = info0.data_type
    npdt = S.NUMPY[dt]
    esz = np.dtype(npdt).itemsize
    start, shape = [int(v) for v in assign.start], [int(v) for v in assign.shape]
    nd = len(shape)
    plane = int(np.prod(shape[1:])) if nd > 1 else 1
    dev0 = H.DeviceBuffer(int(np.prod(shape)) * esz)
    # pieces of about 512 MiB, each chunk decoded once (zarrs_filter._read_pieces)
    pieces = _read_pieces(start, shape, info0.chunk_shape, esz)
    plane2 = int(np.prod(shape[2:])) if nd > 2 else 1
    piece_elems = [(b - a) * (yb - ya) * plane2 if nd >= 2 else (b - a)
                   for a, b, ya, yb in pieces]
    nbuf = min(3, len(pieces))
    bufs = [H.PinnedBuffer(max(piece_elems) * esz) for _ in range(nbuf)]
    evs = [None] * nbuf
    stream = H.Stream()
    phases = {"setup_s": time.perf_counter() - t0, "read_pieces": len(pieces)}

    def decode(k):
        a, b, ya, yb = pieces[k]
        pshape = [b - a, yb - ya] + shape[2:] if nd >= 2 else [b - a]
        pstart = [a, ya] + start[2:] if nd >= 2 else [a]
        h = bufs[k % nbuf].array(npdt, pshape)
        S.read_array(lvl0, pstart, pshape, nthreads=nthreads, out=h)
        return h

    with ThreadPoolExecutor(1) as ex:
        fut = ex.submit(decode, 0)
        for k, (a, b, ya, yb) in enumerate(pieces):
            h = fut.result()
            if k + 1 < len(pieces):
                if evs[(k + 1) % nbuf] is not None:
                    evs[(k + 1) % nbuf].synchronize()  # its last H2D has finished
                fut = ex.submit(decode, k + 1)
            src = ctypes.c_void_p(h.ctypes.data)
            if nd >= 2 and yb - ya < shape[1]:  # the piece's rows land with the box's pitch
                width = (yb - ya) * plane2 * esz
                H.copy2d_async(dev0.at(((a - start[0]) * shape[1] + (ya - start[1])) * plane2 * esz),
                               shape[1] * plane2 * esz, src, width, width, b - a, H.H2D, stream)
            else:  # whole rows: one contiguous copy
                H.copy_async(dev0.at((a - start[0]) * plane * esz), src, (b - a) * plane * esz,
                             H.H2D, stream)
            ev = H.Event()
            ev.record(stream)
            evs[k % nbuf] = ev
    stream.synchronize()
    read_s = time.perf_counter() - t0
    t1 = time.perf_counter()
    L = assign.local_levels
    ctx = F.Context(device)
    shapes = F.pyramid_level_shapes(shape, factor, L)
    outs = [H.DeviceBuffer(int(np.prod(sh)) * esz) for sh in shapes]
    ptrs = (ctypes.c_void_p * max(len(outs), 1))(*[o.ptr.value for o in outs])
    written = ctypes.c_int()
    code = _abi.DTYPES[dt]
    _abi.check(_abi.lib().zt_pyramid_downsample(
        ctx.handle, code, dev0.ptr, _abi.i64_array(shape), nd, _abi.i64_array(factor), int(L),
        int(discrete), ptrs, ctypes.byref(written)))
    levels = [(outs[i], tuple(shapes[i])) for i in range(written.value)]
    while len(levels) < L:  # the box's own stop rule ended early: one level at a time
        src, sshape = levels[-1] if levels else (dev0, tuple(shape))
        oshape = tuple(assign.level_boxes[len(levels)][1])
        o = H.DeviceBuffer(int(np.prod(oshape)) * esz)
        _abi.check(_abi.lib().zt_downsample_apply_ndarray(
            ctx.handle, code, src.ptr, _abi.i64_array(sshape), nd, _abi.i64_array(factor),
            int(discrete), code, o.ptr))
        levels.append((o, oshape))
    ctx.synchronize()
    kernel_s = time.perf_counter() - t1
    t2 = time.perf_counter()
    keep, host = [], []
    for buf, sh in levels:
        pb = H.PinnedBuffer(int(np.prod(sh)) * esz)
        H.copy_async(pb.ptr, buf.ptr, int(np.prod(sh)) * esz, H.D2H, stream)
        keep.append(pb)
        host.append(pb.array(npdt, sh))
    stream.synchronize()
    phases["d2h_s"] = time.perf_counter() - t2
    return host, read_s, kernel_s, keep, phases


def _octant_worker(out_root: str, assign, factor, discrete: bool, device: int, nthreads: int,
                   scratch: str, env=None, compute=None, src0=None) -> dict:
    """One process of `zarrs_ome --gpus N` (SURVEY.md §8(e) octant ownership): read this rank's
    factor^L-aligned level-0 box into HBM, compute levels 1..L of the box there (the windows never
    cross an aligned box boundary), write every output chunk lying wholly inside the box, and
    save the pieces of the chunks that cross box boundaries for the host assembly. `compute`
    (tests only) replaces the device (read box, downsample level) pair."""
    import numpy as _np
    os.environ.update(env or {})
    t0 = time.perf_counter()
    st = {"rank": assign.rank, "read_s": 0.0, "kernel_s": 0.0, "write_s": 0.0, "pieces": [],
          "voxels": 0}
    if assign.coord is None or assign.local_levels == 0:
        return st
    # level 0: the output's copy, or the input itself while the parent is still copying it
    lvl0 = src0 or os.path.join(out_root, "0")
    info0 = S.open_array(lvl0)
    keep = None
    if compute is None and os.environ.get("ZT_NO_TORCH") == "1":
        # a worker of octant_pool: no torch in this process (hiprt.py)
        host, st["read_s"], st["kernel_s"], keep, ph = _box_levels_no_torch(
            lvl0, info0, assign, list(factor), discrete, device, nthreads)
        st.update(ph)
        host_iter = iter(host)
        cur = None
        level, to_host = (lambda x: next(host_iter)), (lambda x: x)
    elif compute is None:
        import torch
        from . import filter as F
        # the box streamed into HBM chunk row by chunk row (decode || H2D)
        cur = read_to_device(lvl0, device, nthreads, start=assign.start, shape=assign.shape)
        st["read_s"] = time.perf_counter() - t0
        t_pyr = time.perf_counter()
        ctx = F.default_context(device)
        ds = F.Downsample(factor, discrete=discrete)
        # levels 1..L of the box in one call: up to three 2x2x2 mean levels per launch
        # (zt_pyramid_downsample, the level-fused kernel), bit-identical to per-level launches
        fused = F.pyramid(cur, factor, max_levels=assign.local_levels, discrete=discrete, ctx=ctx)
        ctx.synchronize()
        st["kernel_s"] = time.perf_counter() - t_pyr
        fused_iter = iter(fused)

        def level(x):
            y = next(fused_iter, None)
            if y is None:  # the box's own stop rule ended early: one level at a time
                y = ds._apply(x, None, discrete, ctx)
                ctx.synchronize()
            return y

        def to_host(x):
            if x.dtype == torch.bfloat16:
                x = x.view(torch.uint16)
            h = torch.empty(tuple(x.shape), dtype=x.dtype, pin_memory=True)
            h.copy_(x)
            return h.numpy()
    else:
        cur = S.read_array(lvl0, assign.start, assign.shape, nthreads=nthreads)
        level, to_host = compute, (lambda x: x)
        st["read_s"] = time.perf_counter() - t0
    for k in range(1, assign.local_levels + 1):
        bstart, bshape = assign.level_boxes[k - 1]
        t1 = time.perf_counter()
        cur = level(cur)
        st["kernel_s"] += time.perf_counter() - t1
        if tuple(cur.shape) != tuple(bshape):
            raise _abi.FilterError(_abi.ERR_OTHER, f"level {k} box {tuple(cur.shape)} != "
                                   f"{tuple(bshape)}")
        t2 = time.perf_counter()
        path = os.path.join(out_root, str(k))
        li = S.open_array(path)
        arr = to_host(cur)
        st["voxels"] += int(arr.size)
        lo, hi, i0, i1 = _box_chunks(bstart, bshape, li.chunk_shape, li.shape)
        if all(b > a for a, b in zip(i0, i1)):
            sl = tuple(slice(a - b, c - b) for a, c, b in zip(i0, i1, bstart))
            S.write_array(path, _np.ascontiguousarray(arr[sl]), i0, nthreads=nthreads)
        # chunks the box only partly covers: this rank's piece of each, assembled by the host
        for idx in _np.ndindex(*[h - l for l, h in zip(lo, hi)]):
            cidx = [l + i for l, i in zip(lo, idx)]
            c0 = [i * c for i, c in zip(cidx, li.chunk_shape)]
            c1 = [min(a + c, s) for a, c, s in zip(c0, li.chunk_shape, li.shape)]
            if all(a >= x and b <= y for a, b, x, y in zip(c0, c1, i0, i1)):
                continue  # written whole above
            p0 = [max(a, b) for a, b in zip(c0, bstart)]
            p1 = [min(a, b + n) for a, b, n in zip(c1, bstart, bshape)]
            if any(b <= a for a, b in zip(p0, p1)):
                continue
            sl = tuple(slice(a - b, c - b) for a, c, b in zip(p0, p1, bstart))
            f = os.path.join(scratch, f"l{k}_r{assign.rank}_{'_'.join(map(str, cidx))}.npy")
            _np.save(f, _np.ascontiguousarray(arr[sl]))
            st["pieces"].append((k, tuple(cidx), tuple(p0), f))
        st["write_s"] += time.perf_counter() - t2
    st["wall_s"] = time.perf_counter() - t0
    st["torch_loaded"] = "torch" in sys.modules
    del keep  # the pinned level buffers, after their last use
    return st


def prepare_octant_levels(out_root: str, level_shapes, local_levels: int, src0=None) -> None:
    """Create the level arrays 1..local_levels (each from the previous level's encoding,
    zarrs_ome.rs:528-560; level 0's encoding from `src0` when given) with their metadata pending
    until every chunk is written."""
    for i in range(1, local_levels + 1):
        src, dst = os.path.join(out_root, str(i - 1)), os.path.join(out_root, str(i))
        if i == 1 and src0:
            src = src0
        S.create_output(src, dst, None, level_shapes[i - 1],
                        level_encoding(S.open_array(src), level_shapes[i - 1]))
        _hold_metadata(dst)


def copy_tree(src: str, dst: str, nthreads: int = 0) -> None:
    """shutil.copytree on a pool of threads: level 0 is a copy of the input (copy_dir,
    zarrs_ome.rs:341-356) of thousands of chunk files, and one thread copying them (in-kernel
    sendfile per file) was the longest phase of a warm-cache zarrs_ome run (2048^3 u16: 2.0-2.4 s
    of 2.6). The files are copied with shutil.copy2, as copytree does; directories first."""
    from concurrent.futures import ThreadPoolExecutor
    files = []
    for root, dirs, names in os.walk(src):
        rel = os.path.relpath(root, src)
        out = dst if rel == "." else os.path.join(dst, rel)
        os.makedirs(out, exist_ok=False if rel == "." else True)
        files.extend((os.path.join(root, n), os.path.join(out, n)) for n in names)
    workers = max(1, nthreads or min(16, os.cpu_count() or 1))
    if workers == 1 or len(files) < 64:
        for a, b in files:
            shutil.copy2(a, b)
        return
    with ThreadPoolExecutor(workers) as ex:
        for _ in ex.map(lambda ab: shutil.copy2(*ab), files, chunksize=16):
            pass


def _octant_warmup(device: int) -> float:
    """Run first on each pre-spawned octant worker (octant_pool): load the HIP library and create
    the device's context while the parent still prepares the levels. The workers run without
    torch (ZT_NO_TORCH=1, hiprt.py), whose import and runtime set-up were most of a small rank's
    time."""
    import ctypes
    n = ctypes.c_int(0)
    _abi.lib().zt_device_count(ctypes.byref(n))
    if 0 <= device < n.value:
        from . import hiprt
        hiprt.set_device(device)
    return time.time()


class OctantPool:
    """The spawned worker processes of run_octants: one single-process executor per rank, warmed
    up on that rank's device, so the rank's octant task runs in the process whose HIP context
    already lives on its device (a shared queue could hand a warmed worker another device's task
    and leave contexts on two devices)."""

    def __init__(self, devices):
        import multiprocessing as mp
        from concurrent.futures import ProcessPoolExecutor
        ctx = mp.get_context("spawn")
        self.devices = list(devices)
        self.execs = [ProcessPoolExecutor(1, mp_context=ctx) for _ in self.devices]
        # the workers never import torch (ZT_NO_TORCH=1 in the environment they are spawned with:
        # a process starts at its first submit, the warm-up, inside this setting)
        old = os.environ.get("ZT_NO_TORCH")
        os.environ["ZT_NO_TORCH"] = "1"
        try:
            for ex, d in zip(self.execs, self.devices):
                ex.submit(_octant_warmup, d)
        finally:
            if old is None:
                os.environ.pop("ZT_NO_TORCH", None)
            else:
                os.environ["ZT_NO_TORCH"] = old

    def submit(self, rank: int, fn, *args):
        """Run fn(*args) in rank's process (rank's device was warmed up there)."""
        return self.execs[rank].submit(fn, *args)

    def shutdown(self, wait: bool = True, cancel_futures: bool = False) -> None:
        for ex in self.execs:
            ex.shutdown(wait=wait, cancel_futures=cancel_futures)


def octant_pool(gpus: int, devices) -> OctantPool:
    """The worker processes of run_octants, started early with a warm-up task each (rank g on
    devices[g]), before this process initialises any device (spawn, not fork)."""
    return OctantPool(list(devices)[:gpus])


def run_octants(out_root: str, shape0, factor, levels, discrete: bool, gpus: int, devices=None,
                nthreads: int = 0, log=print, compute=None, src0=None, pool=None):
    """Levels 1..L of the pyramid over `gpus` processes, one per GPU, each owning a factor^L-
    aligned box of level 0 (shard.octant_assignment; no exchange between processes). The level
    arrays 1..L must exist with pending metadata; chunks crossing box boundaries are assembled
    on the host (shard.assemble_chunk) and written by this (parent) process. `pool`: a process
    pool from octant_pool (the caller shuts it down), else one is spawned here. Returns (L,
    stats)."""
    from . import shard
    assigns = [shard.octant_assignment(g, gpus, shape0, factor, levels) for g in range(gpus)]
    L = assigns[0].local_levels
    devices = list(devices or range(gpus))
    per = max(1, (nthreads or min(16, os.cpu_count() or 1)) // gpus)
    host_share = S.host_available_bytes() // gpus
    envs = [{"ZT_STORE_HOST_MEMORY": str(host_share)} for _ in range(gpus)]
    scratch = tempfile.mkdtemp(prefix=".zt_octants_", dir=out_root)
    t0 = time.perf_counter()
    ex = pool if pool is not None else octant_pool(gpus, devices)
    try:
        try:
            futs = [ex.submit(g, _octant_worker, out_root, assigns[g], list(factor), discrete,
                              devices[g], per, scratch, envs[g], compute, src0)
                    for g in range(gpus) if assigns[g].coord is not None]
            parts = [f.result() for f in futs]
        finally:
            if pool is None:
                ex.shutdown()
        t1 = time.perf_counter()
        # host assembly of the chunks that cross box boundaries
        by_chunk: dict = {}
        for p in parts:
            for k, cidx, p0, f in p["pieces"]:
                by_chunk.setdefault((k, cidx), []).append((p0, f))
        n_assembled = 0
        for (k, cidx), pieces in sorted(by_chunk.items()):
            path = os.path.join(out_root, str(k))
            li = S.open_array(path)
            c0 = [i * c for i, c in zip(cidx, li.chunk_shape)]
            cshape = [min(c, s - a) for a, c, s in zip(c0, li.chunk_shape, li.shape)]
            arrs = [(p0, np.load(f)) for p0, f in pieces]
            if sum(a.size for _, a in arrs) != int(np.prod(cshape)):
                raise _abi.FilterError(_abi.ERR_OTHER, f"level {k} chunk {cidx}: the ranks' "
                                       "pieces do not cover it")
            S.write_array(path, shard.assemble_chunk(c0, cshape, arrs), c0, nthreads=nthreads)
            n_assembled += 1
    finally:
        shutil.rmtree(scratch, ignore_errors=True)
    st = {"wall_s": time.perf_counter() - t0, "assemble_s": time.perf_counter() - t1,
          "processes": len(parts), "assembled_chunks": n_assembled, "local_levels": L,
          "grid": list(assigns[0].grid),
          "per_rank": [{k: v for k, v in p.items() if k != "pieces"} for p in parts]}
    log(f"   levels 1-{L} on {len(parts)} processes (rank grid {list(assigns[0].grid)}): "
        f"{st['wall_s']:.2f}s, {n_assembled} chunks assembled on the host")
    return L, st


def run(input_path, output_path, factor=None, max_levels: int = 10, discrete: bool = False,
        name=None, exists: str = "erase", device: int = 0, nthreads: int = 0,
        gaussian_sigma=None, gaussian_kernel_half_size=None, physical_size=None,
        physical_units=None, group_attributes=None, reencoding=None, log=print,
        device_resident: bool = True, chunk_limit: int = 0, gpus: int = 1,
        gpu_devices=None) -> dict:
    """zarrs_ome (zarrs_ome.rs:156-760). gpus > 1: one process per GPU — without a Gaussian the
    levels are split by octant ownership (run_octants), with one every level is split by output
    chunk rows (zarrs_filter.run_rows_parallel); `gpu_devices` maps process g to a device."""
    t0 = time.perf_counter()
    info = S.open_array(input_path)
    nd = info.ndim
    factor = [2] * nd if factor is None else [int(f) for f in factor]
    if len(factor) != nd:
        raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                     "downsample factor must match the array rank")
    gauss = None
    if gaussian_sigma is not None and not discrete:
        sigma = [float(s) for s in gaussian_sigma]
        half = ([int(h) for h in gaussian_kernel_half_size] if gaussian_kernel_half_size
                else [int(math.ceil(s * 3.0)) for s in sigma])
        if len(sigma) != nd or len(half) != nd:
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         "gaussian sigma / kernel half size must match the rank")
        gauss = (sigma, half)
    for what, v in (("physical size", physical_size), ("physical units", physical_units)):
        if v is not None and len(v) != nd:
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         f"{what} must have one entry per axis")
    if reencoding and reencoding.get("data_type") and reencoding["data_type"] not in S.NUMPY:
        raise _abi.UnsupportedDataType(_abi.ERR_UNSUPPORTED_DATA_TYPE,
                                       f"unsupported data type {reencoding['data_type']}")
    group_attrs = {}
    if group_attributes:
        group_attrs.update(json.loads(group_attributes) if isinstance(group_attributes, str)
                           else group_attributes)
    # octant workers (gpus > 1, no Gaussian) spawned now, so their start-up overlaps this
    # process's preparation; unused (and shut down) if the levels do not take the octant path
    pool = octant_pool(gpus, list(gpu_devices or range(gpus))) if gpus > 1 and gauss is None \
        else None
    try:
        return _run(input_path, output_path, info, nd, factor, max_levels, discrete, name, exists,
                    device, nthreads, gauss, physical_size, physical_units, group_attrs, reencoding,
                    log, device_resident, chunk_limit, gpus, gpu_devices, pool, t0)
    finally:
        if pool is not None:
            # every task is done here; the workers' exit (device teardown, ~0.8 s) need not hold
            # up the caller
            pool.shutdown(wait=False, cancel_futures=True)


def _run(input_path, output_path, info, nd, factor, max_levels, discrete, name, exists, device,
         nthreads, gauss, physical_size, physical_units, group_attrs, reencoding, log,
         device_resident, chunk_limit, gpus, gpu_devices, pool, t0) -> dict:
    """The body of run() once its arguments are checked (`pool`: octant_pool or None)."""
    if os.path.exists(output_path):
        if exists == "exit":
            raise _abi.FilterError(_abi.ERR_OTHER, "Output exists, exiting")
        if exists == "erase":
            shutil.rmtree(output_path)
    os.makedirs(output_path, exist_ok=True)
    lvl0 = os.path.join(output_path, "0")
    # level shapes (downsample.rs:162-168) and the stop rule (:731-737): known from the input
    level_shapes = []
    cur_shape = list(info.shape)
    for _ in range(max_levels):
        cur_shape = [max(s // f, 1) for s, f in zip(cur_shape, factor)]
        level_shapes.append(cur_shape)
        if all(f == 1 or s == 1 for f, s in zip(factor, cur_shape)):
            break
    multi = gpus > 1 and _device_ok(device)
    if pool is not None and not (multi and level_shapes):
        pool.shutdown(wait=True, cancel_futures=True)  # no octant path: release the workers
    dt0 = (reencoding or {}).get("data_type") or info.data_type
    info0 = S.ArrayInfo(lvl0, dt0, tuple(info.shape), info.chunk_shape, info.inner_chunk_shape)
    on_device = (not multi and device_resident and _device_ok(device)
                 and _device_pyramid_fits(info0, gauss, device))
    cur = None  # the previous level in HBM (device-resident pyramid)
    copy_thread, copy_err = None, []
    phases = {}  # wall-clock phases of this call (seconds since its start), for the e2e tools
    if reencoding:
        _reencode_level0(input_path, lvl0, reencoding, nthreads, log, device)
    else:
        if os.path.exists(lvl0):
            shutil.rmtree(lvl0)
        # level 0 is a copy of the input (copy_dir, zarrs_ome.rs:341-356); the device-resident
        # pyramid streams the same input into HBM meanwhile (the copy's reads warm the page
        # cache for it, or the other way round), so level 0 costs one pass over the input
        import threading

        def _copy():
            phases["copy_start"] = time.perf_counter() - t0
            try:
                copy_tree(input_path, lvl0, nthreads)
            except BaseException as e:  # re-raised below
                copy_err.append(e)
            phases["copy_end"] = time.perf_counter() - t0
        copy_thread = threading.Thread(target=_copy)
        copy_thread.start()
        if on_device:
            cur, on_device = _ingest(input_path, device, nthreads, log)
    octants_done = 0  # levels 1..octants_done computed by run_octants
    stats = []
    if multi and gauss is None and level_shapes:
        # octant-owned levels on one process per GPU; without reencoding their level 0 is the
        # input itself, so they start while this process is still copying it to level 0
        from . import shard
        src0 = input_path if not reencoding else lvl0
        devices = list(gpu_devices or range(gpus))[:gpus]
        boxes = [shard.octant_assignment(g, gpus, info.shape, factor, len(level_shapes))
                 for g in range(gpus)]
        big = max(boxes, key=lambda b: int(np.prod(b.shape)))
        box_info = S.ArrayInfo(src0, dt0, tuple(big.shape), (), ())
        # every distinct device must hold its processes' boxes (each with its own count)
        fits = all(_device_pyramid_fits(box_info, None, d, sharing=devices.count(d),
                                        host_share=gpus) for d in sorted(set(devices)))
        phases["octant_checks_done"] = time.perf_counter() - t0
        if not (big.local_levels > 0 and fits) and pool is not None:
            # the octant path is not taken: release the warmed-up workers (and their device
            # contexts) before the row-split processes start
            pool.shutdown(wait=True, cancel_futures=True)
        if big.local_levels > 0 and fits:
            prepare_octant_levels(output_path, level_shapes, big.local_levels, src0)
            octants_done, st_oct = run_octants(output_path, list(info.shape), factor,
                                               len(level_shapes), discrete, gpus, devices,
                                               nthreads, log, src0=src0, pool=pool)
            st_oct["levels"] = octants_done
            stats.append(st_oct)
            phases["octants_done"] = time.perf_counter() - t0
    if copy_thread is not None:
        copy_thread.join()
        phases["copy_joined"] = time.perf_counter() - t0
        if copy_err:
            raise copy_err[0]
        log(f"0: copy {input_path} -> {lvl0} ({info.data_type} {list(info.shape)})")
    if on_device and cur is None:
        cur, on_device = _ingest(lvl0, device, nthreads, log)
    # move array 0's attributes to the group (zarrs_ome.rs:368-377)
    meta0_path = os.path.join(lvl0, "zarr.json")
    with open(meta0_path) as f:
        meta0 = json.load(f)
    moved = dict(meta0.get("attributes") or {})
    moved.pop("_zarrs", None)
    group_attrs.update(moved)
    meta0["attributes"] = {}
    with open(meta0_path, "w") as f:
        json.dump(meta0, f, indent=2)
    dim_names = meta0.get("dimension_names")

    scale = [1.0] * nd
    datasets = [{"path": "0", "coordinateTransformations": [
        {"type": "scale", "scale": list(scale)}]}]
    shape = list(S.open_array(lvl0).shape)
    fused_levels = None  # every level of the device-resident mean / mode pyramid, one call
    if on_device:
        from . import filter as F
        ctx = F.default_context(device)
        if gauss is None:
            # zt_pyramid_downsample: up to three 2x2x2 mean levels per launch (level-fused
            # kernel), bit-identical to the per-level launches
            t1 = time.perf_counter()
            fused_levels = F.pyramid(cur, factor, max_levels=len(level_shapes), discrete=discrete,
                                     ctx=ctx)
            ctx.synchronize()
            t_pyr = time.perf_counter() - t1
            log(f"   levels 1-{len(fused_levels)} on the device in {t_pyr:.3f}s")
    for i in range(1, len(level_shapes) + 1):
        src, dst = os.path.join(output_path, str(i - 1)), os.path.join(output_path, str(i))
        src_info = S.open_array(src)
        out_shape = level_shapes[i - 1]
        enc = level_encoding(src_info, out_shape)
        if i <= octants_done:
            _publish_metadata(dst)
        elif on_device:
            # the level from the previous one in HBM: (Gaussian, f32) then the downsample, the
            # same kernels as the store path's per-row calls (chunked == whole array)
            t1 = time.perf_counter()
            S.create_output(src, dst, None, out_shape, enc)
            _hold_metadata(dst)
            if fused_levels is not None and i <= len(fused_levels):
                nxt = fused_levels[i - 1]
                fused_levels[i - 1] = None
                t_k = t_pyr if i == 1 else 0.0
            else:
                v = cur
                if gauss is not None:
                    v = F.Gaussian(gauss[0], gauss[1]).apply_ndarray(v, dtype_out="float32",
                                                                     ctx=ctx)
                ds = F.Downsample(factor, discrete=discrete)
                nxt = ds._apply(v, src_info.data_type, discrete, ctx)
                nxt = nxt.reshape(out_shape)
                ctx.synchronize()
                t_k = time.perf_counter() - t1
            t2 = time.perf_counter()
            write_from_device(dst, nxt, nthreads)
            _publish_metadata(dst)
            stats.append({"wall_s": time.perf_counter() - t1, "decode_s": 0.0,
                          "encode_s": time.perf_counter() - t2, "h2d_s": 0.0, "kernel_s": t_k,
                          "d2h_s": 0.0, "voxels": int(nxt.numel()), "device_resident": True})
            cur = nxt
        elif multi:
            from .zarrs_filter import run_rows_parallel
            if gauss is not None:
                params = {"stride": factor, "sigma": gauss[0], "kernel_half_size": gauss[1],
                          "encoding": enc, "chunk_limit": chunk_limit}
                nm = "downsample_gaussian"
            else:
                params = {"stride": factor, "discrete": discrete, "encoding": enc,
                          "chunk_limit": chunk_limit}
                nm = "downsample"
            stats.append(run_rows_parallel(nm, src, dst, params, out_shape, gpus,
                                           devices=gpu_devices))
        elif gauss is not None:
            stats.append(S.downsample_gaussian(src, dst, factor, gauss[0], gauss[1],
                                               device=device, encoding=enc,
                                               chunk_limit=chunk_limit))
        else:
            stats.append(S.downsample(src, dst, factor, discrete=discrete, device=device,
                                      encoding=enc, chunk_limit=chunk_limit))
        out = S.open_array(dst)
        scale = level_scale(scale, shape, out.shape)
        datasets.append({"path": str(i), "coordinateTransformations": [
            {"type": "scale", "scale": list(scale)},
            {"type": "translation", "translation": level_translation(scale)}]})
        if i > octants_done:
            log(f"{i}: {list(shape)} -> {list(out.shape)} in {stats[-1]['wall_s']:.2f}s")
        shape = list(out.shape)
    units = physical_units or [None] * nd
    axes = [axis_of(dim_names[k] if dim_names and dim_names[k] is not None else str(k),
                    units[k]) for k in range(nd)]
    ms = {}
    if name is not None:
        ms["name"] = name
    ms["axes"] = axes
    ms["datasets"] = datasets
    if physical_size is not None:
        ms["coordinateTransformations"] = [{"type": "scale",
                                            "scale": [float(x) for x in physical_size]}]
    ms["type"] = "mode" if discrete else ("average" if gauss is None else "gaussian")
    ms["metadata"] = {"description": "Created with zarrs_ome", "repository": "zarrs_tools_amd",
                      "version": VERSION}
    group_attrs["ome"] = {"version": "0.5", "multiscales": [ms]}
    group = {"zarr_format": 3, "node_type": "group", "attributes": group_attrs}
    with open(os.path.join(output_path, "zarr.json"), "w") as f:
        json.dump(group, f, indent=2)
    log(f"Output {output_path} in {time.perf_counter() - t0:.2f}s")
    phases["end"] = time.perf_counter() - t0
    return {"levels": len(level_shapes), "stats": stats,
            "phases": {k: round(v, 3) for k, v in phases.items()}}


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    enc = encoding_of({k: getattr(a, k, None) for k in REENCODE_KEYS})
    try:
        run(a.input, a.output, a.factor, a.max_levels, a.discrete, a.name, a.exists, a.device,
            0, a.gaussian_sigma, a.gaussian_kernel_half_size,
            a.physical_size, a.physical_units, a.group_attributes, enc,
            device_resident=not a.no_device_resident, chunk_limit=a.filter_chunk_limit or 0,
            gpus=a.gpus, gpu_devices=a.gpu_devices)
    except _abi.FilterError as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
