"""``zarrs_filter`` for the on-path filters: guided_filter and downsample over Zarr V3 stores.

Mirrors src/bin/zarrs_filter.rs (LDeakin/zarrs_tools 0.7.2) for the filters this framework
accelerates:

    python -m zarrs_tools_amd.zarrs_filter [--exists erase|exit] [--tmp DIR] [--chunk-limit N]
        [--device D] [RUN_CONFIG.json] [guided-filter IN OUT EPSILON RADIUS [--data-type T]
                                        | downsample IN OUT STRIDE [--discrete] [--data-type T]
                                        | gaussian IN OUT SIGMA KERNEL_HALF_SIZE [--data-type T]]

* subcommand arguments as GuidedFilterArguments (guided_filter.rs:25-33),
  DownsampleArguments (downsample.rs:20-33, STRIDE comma delimited) and GaussianArguments
  (gaussian.rs:22-30, SIGMA and KERNEL_HALF_SIZE comma delimited, one entry per axis);
* a JSON run config is a list of {"filter": "guided_filter" | "downsample", "input", "output",
  ...args, "data_type"}, with "$name" meaning a named temporary array under --tmp and an omitted
  input meaning the previous filter's output (zarrs_filter.rs:106-138, :338-381);
* a chain of steps linked only through temporaries (a "$name" or implicit output read by the
  next step alone) runs device-resident when its arrays fit 80 % of the free device memory: the
  chain input is read once, every step runs on the arrays in HBM, the last output is written
  once; the temporaries' zarr.json are created as the store path would create them, but their
  chunks never go through the store (`--no-device-chain` forces the store path);
* every filter takes the reencoding arguments (ZarrReencodingArgs, lib.rs:274-377: -d/--data-type,
  -f/--fill-value, --separator, -c/--chunk-shape, -s/--shard-shape, --array-to-array-codecs,
  --array-to-bytes-codec, --bytes-to-bytes-codecs, --dimension-names, --attributes,
  --attributes-append; the same snake_case keys in a run config), applied to the output array as
  get_array_builder_reencode does (lib.rs:408-650; host/zt_store.cpp build_output);
* `--exists erase` (default) overwrites an existing output, `exit` refuses it (:228-235);
* the output metadata is erased before a filter runs and written when it finishes (:297-313);
* per-chunk progress (Progress, progress.rs:15-119) is shown on a terminal as
  `step/steps rw:READ/WRITE p:PROCESS` (thread-seconds, device seconds), like zarrs_filter.rs:
  149-172.

Filters outside the accelerated path (reencode, crop, rescale, clamp, equal, replace_value,
gradient_magnitude, summed_area_table) are rejected with FilterError::Other: they are out of scope
(DESIGN.md §1). `--chunk-limit N` bounds the chunks in flight (decoded input rows + output rows
being computed or encoded, and the host worker threads) at N, down to the pipeline's unit of one
slab and one output row (guided_filter.rs:251-258); independently the rows held in memory are
bounded by 80 % of the available host and device memory, failing like calculate_chunk_limit
(filter.rs:52-66) when not even one row fits.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

from . import _abi
from . import store as S

ON_PATH = ("guided_filter", "downsample", "gaussian")


def _parse_stride(s: str):
    return [int(x) for x in s.split(",") if x.strip()]


def _parse_floats(s: str):
    return [float(x) for x in s.split(",") if x.strip()]


# ZarrReencodingArgs (lib.rs:274-377), flattened into every filter's arguments
# (filter_common_arguments.rs:7-16) and into the JSON run config (serde flatten).
REENCODE_KEYS = ("data_type", "fill_value", "separator", "chunk_shape", "shard_shape",
                 "array_to_array_codecs", "array_to_bytes_codec", "bytes_to_bytes_codecs",
                 "dimension_names", "attributes", "attributes_append")


def _parse_fill_value(s: str):
    """parse_fill_value: JSON (0, 100, -1.5, "NaN", "[0, 255]"), else the bare string."""
    if s in ("NaN", "Infinity", "-Infinity"):
        return s  # the Zarr V3 fill-value strings, kept as strings
    try:
        return json.loads(s)
    except ValueError:
        return s


def _add_reencode_args(p: argparse.ArgumentParser) -> None:
    p.add_argument("-d", "--data-type", default=None)
    p.add_argument("-f", "--fill-value", type=_parse_fill_value, default=None)
    p.add_argument("--separator", default=None, choices=["/", "."])
    p.add_argument("-c", "--chunk-shape", type=_parse_stride, default=None)
    p.add_argument("-s", "--shard-shape", type=_parse_stride, default=None)
    p.add_argument("--array-to-array-codecs", default=None)
    p.add_argument("--array-to-bytes-codec", default=None)
    p.add_argument("--bytes-to-bytes-codecs", default=None)
    p.add_argument("--dimension-names", type=lambda s: s.split(","), default=None)
    p.add_argument("--attributes", default=None)
    p.add_argument("--attributes-append", default=None)
    p.add_argument("--chunk-limit", dest="filter_chunk_limit", type=int, default=None)


def _reencode_of(a) -> dict:
    return {k: getattr(a, k) for k in REENCODE_KEYS if getattr(a, k, None) is not None}


def encoding_of(step: dict) -> dict | None:
    """The reencoding arguments of a run-config step (JSON strings of the codec / attribute
    arguments parsed), or None when it has none."""
    enc = {}
    for k in REENCODE_KEYS:
        v = step.get(k)
        if v is None:
            continue
        if k in ("array_to_array_codecs", "array_to_bytes_codec", "bytes_to_bytes_codecs",
                 "attributes", "attributes_append") and isinstance(v, str):
            v = json.loads(v)
        if k in ("chunk_shape", "shard_shape") and isinstance(v, str):
            v = _parse_stride(v)
        enc[k] = v
    return enc or None


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="zarrs_filter",
                                 description="Apply filters to a Zarr V3 array on an MI355X.")
    ap.add_argument("--exists", choices=["erase", "exit"], default="erase")
    ap.add_argument("--tmp", default=None, help="directory for temporary ($name) arrays")
    ap.add_argument("--chunk-limit", type=int, default=None)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--stats", action="store_true", help="print per-filter stats as JSON")
    ap.add_argument("--gpus", type=int, default=1,
                    help="split every store step over this many GPUs (one process each) by "
                         "output chunk rows")
    ap.add_argument("--no-device-chain", action="store_true",
                    help="run every step store -> store, also chains of temporaries")
    sub = ap.add_subparsers(dest="filter")
    g = sub.add_parser("guided-filter", help="Apply a guided filter (edge preserving noise filter).")
    g.add_argument("input")
    g.add_argument("output")
    g.add_argument("epsilon", type=float)
    g.add_argument("radius", type=int)
    _add_reencode_args(g)
    d = sub.add_parser("downsample", help="Downsample an image given a stride.")
    d.add_argument("input")
    d.add_argument("output")
    d.add_argument("stride", type=_parse_stride)
    d.add_argument("--discrete", action="store_true")
    _add_reencode_args(d)
    gs = sub.add_parser("gaussian", help="Apply a Gaussian kernel.")
    gs.add_argument("input")
    gs.add_argument("output")
    gs.add_argument("sigma", type=_parse_floats)
    gs.add_argument("kernel_half_size", type=_parse_stride)
    _add_reencode_args(gs)
    return ap


def _steps_from_cli(a) -> list:
    if a.filter == "guided-filter":
        return [{"filter": "guided_filter", "input": a.input, "output": a.output,
                 "epsilon": a.epsilon, "radius": a.radius, "data_type": a.data_type,
                 "chunk_limit": a.filter_chunk_limit, **_reencode_of(a)}]
    if a.filter == "downsample":
        return [{"filter": "downsample", "input": a.input, "output": a.output,
                 "stride": a.stride, "discrete": a.discrete, "data_type": a.data_type,
                 "chunk_limit": a.filter_chunk_limit, **_reencode_of(a)}]
    if a.filter == "gaussian":
        return [{"filter": "gaussian", "input": a.input, "output": a.output, "sigma": a.sigma,
                 "kernel_half_size": a.kernel_half_size, "data_type": a.data_type,
                 "chunk_limit": a.filter_chunk_limit, **_reencode_of(a)}]
    return []


def _is_temp(p) -> bool:
    return p is None or (isinstance(p, str) and p.startswith("$"))


def plan_chains(steps: list) -> list:
    """Maximal runs [i, j] of steps (j > i) where every step before j hands its output to the next
    step only: the output is a temporary (a "$name", or omitted) and the next step reads it (its
    input is that "$name", or omitted = the previous output), and no other step names it."""
    refs: dict = {}
    for st in steps:
        for key in ("input", "output"):
            v = st.get(key)
            if isinstance(v, str) and v.startswith("$"):
                refs[v] = refs.get(v, 0) + 1

    def linked(k):
        out, nxt = steps[k].get("output"), steps[k + 1].get("input")
        if not _is_temp(out):
            return False
        if out is None:
            return nxt is None
        return nxt in (out, None) and refs.get(out, 0) == (2 if nxt == out else 1)

    chains, i = [], 0
    while i < len(steps):
        j = i
        while j + 1 < len(steps) and linked(j):
            j += 1
        if j > i:
            chains.append((i, j))
        i = j + 1
    return chains


def _step_params(step, info):
    """(filter object, output shape, output data type) of a run-config step on an input array."""
    from . import filter as F
    name = step.get("filter")
    dt = step.get("data_type") or (encoding_of(step) or {}).get("data_type") or info.data_type
    if name == "guided_filter":
        if "epsilon" not in step or "radius" not in step:
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         "guided_filter needs epsilon and radius")
        return F.GuidedFilter(float(step["epsilon"]), int(step["radius"])), tuple(info.shape), dt
    if name == "gaussian":
        sigma, half = step.get("sigma"), step.get("kernel_half_size")
        sigma = _parse_floats(sigma) if isinstance(sigma, str) else sigma
        half = _parse_stride(half) if isinstance(half, str) else half
        if not sigma or not half or len(sigma) != info.ndim or len(half) != info.ndim:
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         "gaussian sigma and kernel_half_size need one entry "
                                         "per axis")
        return F.Gaussian(sigma, half), tuple(info.shape), dt
    stride = step.get("stride")
    stride = _parse_stride(stride) if isinstance(stride, str) else stride
    if not stride or len(stride) != info.ndim:
        raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                     "downsample stride must match the array rank")
    f = F.Downsample(stride, discrete=bool(step.get("discrete", False)))
    return f, f.output_shape(info.shape), dt


def _nbytes(shape, data_type) -> int:
    n = 1
    for s in shape:
        n *= int(s)
    return n * S.NUMPY[data_type]().itemsize


def allocation_refused(e: BaseException) -> bool:
    """True for a refused device or pinned-host allocation (the callers then fall back to the
    store -> store path); False for everything else, FilterError (storage, codecs) included."""
    import torch
    if isinstance(e, _abi.FilterError):
        return False
    if isinstance(e, torch.cuda.OutOfMemoryError):
        return True
    msg = str(e).lower()
    return isinstance(e, RuntimeError) and ("out of memory" in msg or "pinned" in msg or
                                            "hiphostmalloc" in msg or "cudahostalloc" in msg)


def _row_spans(start0: int, n0: int, chunk0: int) -> list:
    """[a, b) pieces of the axis-0 range [start0, start0 + n0) cut at the chunk grid, so that
    every chunk (or shard) is decoded / encoded by one piece only."""
    spans, a, end = [], start0, start0 + n0
    while a < end:
        b = min((a // chunk0 + 1) * chunk0, end)
        spans.append((a, b))
        a = b
    return spans


def _read_pieces(start, shape, chunk_shape, esz: int) -> list:
    """The pieces a box read is pipelined in: chunk rows of axis 0, cut along axis 1 at the chunk
    grid into pieces of about ZT_READ_PIECE_KB (default 512 MiB; 0: whole rows). Each chunk is
    still decoded once, but a pinned buffer holds a piece instead of a whole chunk row: pinning
    three 2 GB rows per process made 2048^3 u16 box reads 2x slower
    (profiles/r04_octant_workers*.json). [(a, b, ya, yb)]; ya, yb = 0, 1 for 1-D arrays."""
    nd = len(shape)
    spans = _row_spans(start[0], shape[0], int(chunk_shape[0])) if shape[0] > 0 else []
    if nd < 2:
        return [(a, b, 0, 1) for a, b in spans]
    target = int(os.environ.get("ZT_READ_PIECE_KB", "524288")) << 10
    plane2 = int(np.prod(shape[2:])) if nd > 2 else 1
    cy = int(chunk_shape[1])
    out = []
    for a, b in spans:
        if target > 0:
            m = max(1, target // max(1, (b - a) * cy * plane2 * esz))
            out += [(a, b, ya, yb) for ya, yb in _row_spans(start[1], shape[1], cy * m)]
        else:
            out.append((a, b, start[1], start[1] + shape[1]))
    return out


def read_to_device(path, device: int, nthreads: int = 0, start=None, shape=None):
    """The box [start, start + shape) of a store array (the whole array by default) decoded into
    HBM, overlapped chunk row by chunk row: a host thread decodes row k+1
    into one of three pinned row buffers while row k is copied host-to-device on a side stream
    (the reference copies level 0 then streams it chunk by chunk, zarrs_ome.rs:341-366,
    631-714). Each chunk is decoded once. bfloat16 arrays come back as torch.bfloat16."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from . import filter as F
    info = S.open_array(path)
    nd = info.ndim
    start = [0] * nd if start is None else [int(v) for v in start]
    shape = list(info.shape) if shape is None else [int(v) for v in shape]
    store_dt = "uint16" if info.data_type == "bfloat16" else info.data_type
    tdt = F.torch_dtype(store_dt)
    dev = torch.device("cuda", device)
    x = torch.empty(tuple(shape), dtype=tdt, device=dev)
    if all(v > 0 for v in shape):
        pieces = _read_pieces(start, shape, info.chunk_shape, x.element_size())

        def pshape(p):
            a, b, ya, yb = p
            return [b - a, yb - ya] + shape[2:] if nd >= 2 else [b - a]

        n_max = max(int(np.prod(pshape(p))) for p in pieces)
        nbuf = min(3, len(pieces))
        bufs = [torch.empty((n_max,), dtype=tdt, pin_memory=True) for _ in range(nbuf)]
        evs = [None] * nbuf
        stream = torch.cuda.Stream(device=dev)
        # x was allocated on the caller's current stream: order the copies after any work that
        # stream still has queued on the block the caching allocator handed back
        stream.wait_stream(torch.cuda.current_stream(dev))

        def decode(k):
            a, b, ya, yb = pieces[k]
            ps = pshape(pieces[k])
            h = bufs[k % nbuf][:int(np.prod(ps))].view(ps)
            S.read_array(path, [a, ya] + start[2:] if nd >= 2 else [a], ps, nthreads=nthreads,
                         out=h.numpy())
            return h

        with ThreadPoolExecutor(1) as ex:
            fut = ex.submit(decode, 0)
            for k, (a, b, ya, yb) in enumerate(pieces):
                h = fut.result()
                if k + 1 < len(pieces):
                    ev = evs[(k + 1) % nbuf]
                    if ev is not None:
                        ev.synchronize()  # the H2D that last read this buffer has finished
                    fut = ex.submit(decode, k + 1)
                with torch.cuda.stream(stream):
                    if nd >= 2:
                        x[a - start[0]:b - start[0], ya - start[1]:yb - start[1]].copy_(
                            h, non_blocking=True)
                    else:
                        x[a - start[0]:b - start[0]].copy_(h, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(stream)
                evs[k % nbuf] = ev
        stream.synchronize()
    return x.view(torch.bfloat16) if info.data_type == "bfloat16" else x


def write_from_device(path, x, nthreads: int = 0, start=None) -> None:
    """A device tensor (the box at `start`, default the whole array at `path`) into the store,
    overlapped chunk row by chunk row: row k+1 is copied device-to-host into one of two pinned
    buffers while a host thread encodes row k."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    if x.dtype == torch.bfloat16:
        x = x.view(torch.uint16)
    info = S.open_array(path)
    nd = x.dim()
    start = [0] * nd if start is None else [int(v) for v in start]
    shape = list(x.shape)
    if not shape or any(v == 0 for v in shape):
        return
    spans = _row_spans(start[0], shape[0], int(info.chunk_shape[0]))
    plane = int(np.prod(shape[1:])) if nd > 1 else 1
    rows = max(b - a for a, b in spans)
    nbuf = min(2, len(spans))
    bufs = [torch.empty((rows * plane,), dtype=x.dtype, pin_memory=True) for _ in range(nbuf)]
    futs = [None] * nbuf
    with ThreadPoolExecutor(1) as ex:
        for k, (a, b) in enumerate(spans):
            if futs[k % nbuf] is not None:
                futs[k % nbuf].result()  # this buffer's previous row is encoded
            h = bufs[k % nbuf][:(b - a) * plane].view([b - a] + shape[1:])
            h.copy_(x[a - start[0]:b - start[0]])
            futs[k % nbuf] = ex.submit(S.write_array, path, h.numpy(), [a] + start[1:], nthreads)
        for f in futs:
            if f is not None:
                f.result()


def run_device_chain(steps: list, paths: list, device: int = 0, nthreads: int = 0,
                     log=print, budget_frac: float = 0.8):
    """Run steps[0..] device-resident: paths[k] is step k's input path (paths[k+1] its output).
    Creates every output array as the store path would (S.create_output), reads paths[0] once,
    applies the filters on HBM arrays, writes the last output once. Returns per-step stats, or
    None (nothing done) when the chain's arrays do not fit `budget_frac` of the free device
    memory, in which case the caller runs it store -> store."""
    import torch
    from . import filter as F
    # shapes / types of every array of the chain (metadata only)
    plan, info = [], S.open_array(paths[0])
    peak = 0
    for k, step in enumerate(steps):
        f, oshape, odt = _step_params(step, info)
        peak = max(peak, _nbytes(info.shape, info.data_type) + _nbytes(oshape, odt))
        plan.append((f, info, oshape, odt))
        info = S.ArrayInfo(paths[k + 1], odt, tuple(oshape), info.chunk_shape,
                           info.inner_chunk_shape)
    free, _total = torch.cuda.mem_get_info(device)
    if 2 * peak > budget_frac * free:  # in + out of a step, plus filter scratch of the same order
        return None
    # the chain input and the last output each pass through one pinned host buffer
    src0 = S.open_array(paths[0])
    host_need = max(_nbytes(src0.shape, src0.data_type), _nbytes(plan[-1][2], plan[-1][3]))
    if host_need > budget_frac * S.host_available_bytes():
        return None
    results = []
    t0 = time.perf_counter()
    src_info = S.open_array(paths[0])
    try:
        x = read_to_device(paths[0], device, nthreads)
    except RuntimeError as e:
        if not allocation_refused(e):
            raise  # storage / codec errors (FilterError) are real failures
        return None  # pinned host or device allocation refused: the store path instead
    t_read = time.perf_counter() - t0
    for k, step in enumerate(steps):
        f, src_info_k, oshape, odt = plan[k]
        S.create_output(paths[k], paths[k + 1], odt, oshape, encoding_of(step))
    # The last output is "not finished" (no zarr.json, zarrs_filter.rs:297-313) until its chunks
    # are written; a failing step leaves no output that looks complete. Held only once the input
    # is on the device, so a fallback to the store path never leaves a stale pending file.
    S.hold_metadata(paths[-1])
    dev = torch.device("cuda", device)
    x_dt, x_chunk = src_info.data_type, src_info.chunk_shape
    ctx = F.default_context(device)
    for k, step in enumerate(steps):
        f = plan[k][0]
        out_info = S.open_array(paths[k + 1])
        y = torch.empty(tuple(out_info.shape), dtype=F.torch_dtype(out_info.data_type), device=dev)
        t1 = time.perf_counter()
        f.apply(F.DeviceArray(x, x_chunk, x_dt), F.DeviceArray(y, out_info.chunk_shape,
                                                              out_info.data_type), ctx=ctx)
        ctx.synchronize()
        t_k = time.perf_counter() - t1
        log(f"{k}: {step.get('filter')} device-resident {list(x.shape)} {x_dt} -> "
            f"{list(y.shape)} {out_info.data_type} in {t_k:.3f}s")
        results.append({"wall_s": t_k, "decode_s": t_read if k == 0 else 0.0, "encode_s": 0.0,
                        "h2d_s": 0.0, "kernel_s": t_k, "d2h_s": 0.0, "bytes_read": 0,
                        "bytes_written": 0, "voxels": int(y.numel()), "rows": 0,
                        "threads": nthreads, "device_resident": True})
        x, x_dt, x_chunk = y, out_info.data_type, out_info.chunk_shape
    t2 = time.perf_counter()
    write_from_device(paths[-1], x, nthreads)
    S.publish_metadata(paths[-1])  # finished
    results[-1]["encode_s"] = time.perf_counter() - t2
    return results


def _rows_worker(name: str, src: str, dst: str, params: dict, device: int, rows, nthreads: int,
                 env=None):
    """One process of a multi-GPU store step: output chunk rows [rows[0], rows[1]) on `device`,
    no metadata writes (the parent writes zarr.json once every row is done). `env`: the memory
    budget of this process (ZT_STORE_HOST_MEMORY / ZT_STORE_DEVICE_MEMORY, its share)."""
    os.environ.update(env or {})
    cols = None
    if isinstance(rows, tuple) and len(rows) == 2 and isinstance(rows[0], tuple):
        rows, cols = rows  # ((row range), (column range)): a (t, z) block
    kw = dict(device=device, rows=rows, nthreads=nthreads, erase=False, finish=False,
              encoding=params.get("encoding"), data_type=params.get("data_type"),
              chunk_limit=params.get("chunk_limit") or 0)
    if name == "guided_filter":
        return S.guided_filter(src, dst, params["epsilon"], params["radius"], cols=cols, **kw)
    if name == "gaussian":
        return S.gaussian(src, dst, params["sigma"], params["kernel_half_size"], **kw)
    if name == "downsample_gaussian":  # a zarrs_ome level with --gaussian-sigma
        return S.downsample_gaussian(src, dst, params["stride"], params["sigma"],
                                     params["kernel_half_size"], **kw)
    return S.downsample(src, dst, params["stride"], discrete=params["discrete"], **kw)


def run_rows_parallel(name: str, src: str, dst: str, params: dict, out_shape, gpus: int,
                      nthreads: int = 0, devices=None) -> dict:
    """A store step split over `gpus` processes (one per GPU, guided_filter.rs:260-316's chunk
    loop partitioned into contiguous output chunk rows along axis 0; no data exchange: each
    process reads its rows' inputs with their halo). The output's zarr.json is written once, by
    the parent, after every process finished (zarrs_filter.rs:297-313). `devices` maps process
    g to a device (default g; a 1-GPU rehearsal passes [0] * gpus)."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    info = S.open_array(src)
    S.create_output(src, dst, params.get("data_type"), out_shape, params.get("encoding"))
    out = S.open_array(dst)
    os.remove(os.path.join(dst, "zarr.json"))  # "not finished" until every row is written
    nrows = -(-out.shape[0] // out.chunk_shape[0])
    bounds = [(g * nrows // gpus, (g + 1) * nrows // gpus) for g in range(gpus)]
    if name == "guided_filter" and len(out.shape) >= 4 and gpus > 1:
        # 4-D series (config T): (t, z) blocks of whole chunks that minimise the input the
        # processes decode and filter in all, halo included (shard.block_split): rows along t
        # alone would make each process decode 3x its output timepoints
        from . import shard
        halo = (2 * int(params["radius"])) & 0xFF
        groups = shard.block_split(gpus, out.shape, out.chunk_shape, halo)
        if groups[1] > 1:
            ncol = -(-out.shape[1] // out.chunk_shape[1])
            bounds = []
            for g in range(gpus):
                k0, k1 = g // groups[1], g % groups[1]
                bounds.append(((k0 * nrows // groups[0], (k0 + 1) * nrows // groups[0]),
                               (k1 * ncol // groups[1], (k1 + 1) * ncol // groups[1])))
    devices = devices or list(range(gpus))
    per = max(1, (nthreads or min(16, os.cpu_count() or 1)) // gpus)
    params = dict(params)
    if params.get("chunk_limit"):  # the reference's limit is per process: split it N ways
        params["chunk_limit"] = max(1, int(params["chunk_limit"]) // gpus)
    # each process budgets its share of host memory, and of device memory where processes share
    # a device (a one-GPU rehearsal), so N processes never reserve N x 80 % together
    host_share = S.host_available_bytes() // gpus
    sharing = {d: devices[:gpus].count(d) for d in set(devices[:gpus])}
    envs = []
    for g in range(gpus):
        env = {"ZT_STORE_HOST_MEMORY": str(host_share)}
        if sharing[devices[g]] > 1 and "ZT_STORE_DEVICE_MEMORY" not in os.environ:
            import torch
            free, _ = torch.cuda.mem_get_info(devices[g])
            env["ZT_STORE_DEVICE_MEMORY"] = str(free // sharing[devices[g]])
        envs.append(env)
    t0 = time.perf_counter()
    with ProcessPoolExecutor(gpus, mp_context=mp.get_context("spawn")) as ex:
        def nonempty(b):
            if isinstance(b[0], tuple):
                return b[0][1] > b[0][0] and b[1][1] > b[1][0]
            return b[1] > b[0]
        futs = [ex.submit(_rows_worker, name, src, dst, params, devices[g], bounds[g], per,
                          envs[g])
                for g in range(gpus) if nonempty(bounds[g])]
        parts = [f.result() for f in futs]
    S.create_output(src, dst, params.get("data_type"), out_shape, params.get("encoding"))
    st = {k: sum(p[k] for p in parts) for k in parts[0] if isinstance(parts[0][k], (int, float))}
    st["wall_s"] = time.perf_counter() - t0
    st["processes"] = len(parts)
    del info
    return st


def _device_ok(device: int) -> bool:
    try:
        import torch
        return torch.cuda.is_available() and device < torch.cuda.device_count()
    except Exception:
        return False


def run(steps: list, exists: str = "erase", tmp: str | None = None,
        chunk_limit: int | None = None, device: int = 0, stats: bool = False,
        log=print, device_chain: bool = True, gpus: int = 1, gpu_devices=None) -> list:
    """Run a list of filter steps (the run-config form); returns the per-step stats. gpus > 1:
    every store step is split over that many processes by output chunk rows (one per GPU;
    `gpu_devices` maps process g to a device, default g); device-resident chains are then off."""
    if gpus > 1:
        device_chain = False
    tmp_root = tmp or tempfile.gettempdir()
    temps: dict[str, str] = {}
    made: list[str] = []
    last_output = None
    results = []

    def resolve(p, what):
        if p is None:
            if what == "input" and last_output is not None:
                return last_output
            if what == "output":
                d = tempfile.mkdtemp(prefix="zt_", dir=tmp_root)
                made.append(d)
                return d
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         "the first filter needs an input")
        if isinstance(p, str) and p.startswith("$"):
            if p not in temps:
                temps[p] = tempfile.mkdtemp(prefix=p[1:] + "_", dir=tmp_root)
                made.append(temps[p])
            return temps[p]
        return p

    def prepare(dst):
        if exists == "exit" and os.path.exists(os.path.join(dst, "zarr.json")):
            raise _abi.FilterError(_abi.ERR_OTHER, f"output {dst} already exists")
        if os.path.isdir(dst) and dst not in made:
            # create_array erases the output prefix (zarrs_filter.rs:76); only the
            # temporaries this run just made (empty) are kept
            shutil.rmtree(dst)

    def store_step(i, step, src, dst):
        name = step.get("filter")
        limit = step.get("chunk_limit") or chunk_limit or 0  # chunks in flight, not threads
        info = S.open_array(src)
        f, out_shape, _dt = _step_params(step, info)
        enc = encoding_of(step)
        if name == "guided_filter":
            params = {"epsilon": float(step["epsilon"]), "radius": int(step["radius"])}
            log(f"{i}: guided_filter epsilon={params['epsilon']} radius={params['radius']} "
                f"{src} ({info.data_type} {list(info.shape)}) -> {dst}")
        elif name == "gaussian":
            params = {"sigma": list(f.sigma), "kernel_half_size": list(f.kernel_half_size())}
            log(f"{i}: gaussian sigma={params['sigma']} "
                f"kernel_half_size={params['kernel_half_size']} "
                f"{src} ({info.data_type} {list(info.shape)}) -> {dst}")
        else:
            params = {"stride": list(f.stride), "discrete": bool(step.get("discrete", False))}
            log(f"{i}: downsample stride={params['stride']} discrete={params['discrete']} "
                f"{src} ({info.data_type} {list(info.shape)}) -> {dst}")
        params.update(data_type=step.get("data_type"), encoding=enc, chunk_limit=limit)
        if gpus > 1:
            st = run_rows_parallel(name, src, dst, params, out_shape, gpus, 0,
                                   devices=gpu_devices)
        elif name == "guided_filter":
            st = S.guided_filter(src, dst, params["epsilon"], params["radius"],
                                 data_type=params["data_type"], device=device,
                                 encoding=enc, chunk_limit=limit)
        elif name == "gaussian":
            st = S.gaussian(src, dst, params["sigma"], params["kernel_half_size"],
                            data_type=params["data_type"], device=device, encoding=enc,
                            chunk_limit=limit)
        else:
            st = S.downsample(src, dst, params["stride"], discrete=params["discrete"],
                              data_type=params["data_type"], device=device, encoding=enc,
                              chunk_limit=limit)
        out = S.open_array(dst)
        log(f"   -> {out.data_type} {list(out.shape)} in {st['wall_s']:.2f}s "
            f"(rw:{st['decode_s']:.2f}/{st['encode_s']:.2f} p:{st['kernel_s']:.3f})")
        if stats:
            log(json.dumps({"step": i, "filter": name, **st}))
        return st

    for step in steps:
        name = step.get("filter")
        if name not in ON_PATH:
            raise _abi.FilterError(_abi.ERR_OTHER,
                                   f"filter {name!r} is outside the accelerated path "
                                   f"(supported: {', '.join(ON_PATH)})")
    chains = dict(plan_chains(steps)) if device_chain and _device_ok(device) else {}
    t_all = time.perf_counter()
    if sys.stderr.isatty():
        def _show(p):
            sys.stderr.write(f"\r  {p['step']}/{p['num_steps']} rw:{p['read_s']:.2f}/"
                             f"{p['write_s']:.2f} p:{p['process_s']:.3f}")
            if p["step"] == p["num_steps"]:
                sys.stderr.write("\n")
            sys.stderr.flush()
        S.set_progress_callback(_show)
    try:
        i = 0
        while i < len(steps):
            j = chains.get(i, i)
            paths = [resolve(steps[i].get("input"), "input")]
            for k in range(i, j + 1):
                d = resolve(steps[k].get("output"), "output")
                prepare(d)
                paths.append(d)
                last_output = d
            res = None
            if j > i:
                threads = chunk_limit or 0
                res = run_device_chain(steps[i:j + 1], paths, device, threads, log)
                if res is not None and stats:
                    for k, st in enumerate(res):
                        log(json.dumps({"step": i + k, "filter": steps[i + k].get("filter"), **st}))
            if res is None:  # one step, or a chain too large for the device: store -> store
                res = [store_step(k, steps[k], paths[k - i], paths[k - i + 1])
                       for k in range(i, j + 1)]
            results.extend(res)
            i = j + 1
    finally:
        if sys.stderr.isatty():
            S.set_progress_callback(None)
        for d in made:
            shutil.rmtree(d, ignore_errors=True)
    log(f"Completed in {time.perf_counter() - t_all:.2f}s")
    return results


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    config = None
    # a leading positional JSON run config (Cli::run_config), before any subcommand
    if argv and argv[0].endswith(".json") and os.path.exists(argv[0]):
        config = argv.pop(0)
    a = build_parser().parse_args(argv)
    if config:
        with open(config) as f:
            steps = json.load(f)
        if isinstance(steps, dict):
            steps = [steps]
    else:
        steps = _steps_from_cli(a)
    if not steps:
        build_parser().print_help()
        return 2
    try:
        run(steps, a.exists, a.tmp, a.chunk_limit, a.device, a.stats,
            device_chain=not a.no_device_chain, gpus=a.gpus)
    except _abi.FilterError as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
