"""Zarr V3 filesystem arrays and the store -> store filters (host side of the C ABI).

Mirrors what the reference does through zarrs (0.20.0-beta.2): ``load_array`` / ``create_array``
in src/bin/zarrs_filter.rs:63-87, the filters' ``apply`` over Array<FilesystemStore>
(guided_filter.rs:240-319, downsample.rs:170-286) and zarrs_ome's level loop
(zarrs_ome.rs:515-738). All I/O and compute run in libzarrs_tools_amd.so; this module only
marshals arguments (numpy is used for host buffers in tests and tools).
"""
from __future__ import annotations

import ctypes
import json
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _abi
from ._abi import DTYPES, DTYPE_NAMES, check, i64_array, lib

NUMPY = {
    "bool": np.bool_, "int8": np.int8, "int16": np.int16, "int32": np.int32, "int64": np.int64,
    "uint8": np.uint8, "uint16": np.uint16, "uint32": np.uint32, "uint64": np.uint64,
    "bfloat16": np.uint16, "float16": np.float16, "float32": np.float32, "float64": np.float64,
}

SYNTH_STEP_NOISE_F32 = 0
SYNTH_U16 = 1
SEED = 0x5EED2025


def _b(path) -> bytes:
    return os.fspath(path).encode()


def _dt(dtype) -> int:
    if dtype is None:
        return -1
    if isinstance(dtype, int):
        return dtype
    if dtype not in DTYPES:
        raise _abi.UnsupportedDataType(_abi.ERR_UNSUPPORTED_DATA_TYPE,
                                       f"unsupported data type {dtype}")
    return DTYPES[dtype]


@dataclass
class ArrayInfo:
    path: str
    data_type: str
    shape: tuple
    chunk_shape: tuple
    inner_chunk_shape: tuple

    @property
    def ndim(self) -> int:
        return len(self.shape)

    @property
    def metadata(self) -> dict:
        with open(os.path.join(self.path, "zarr.json")) as f:
            return json.load(f)


def open_array(path) -> ArrayInfo:
    """Array::open on a filesystem store (zarr.json V3)."""
    dt, nd = ctypes.c_int(), ctypes.c_int()
    shp, ch, inner = (ctypes.c_int64 * 8)(), (ctypes.c_int64 * 8)(), (ctypes.c_int64 * 8)()
    check(lib().zt_store_array_info(_b(path), ctypes.byref(dt), ctypes.byref(nd), shp, ch, inner))
    n = nd.value
    return ArrayInfo(os.fspath(path), DTYPE_NAMES[dt.value], tuple(shp[:n]), tuple(ch[:n]),
                     tuple(inner[:n]))


def codecs_json(compression: Optional[str] = None, level: int = 1,
                shard_inner: Optional[Sequence[int]] = None) -> Optional[str]:
    """A Zarr V3 codec list: bytes (+ gzip/zstd), optionally inside sharding_indexed."""
    chain = [{"name": "bytes", "configuration": {"endian": "little"}}]
    if compression == "gzip":
        chain.append({"name": "gzip", "configuration": {"level": int(level)}})
    elif compression == "zstd":
        chain.append({"name": "zstd", "configuration": {"level": int(level), "checksum": False}})
    elif compression not in (None, "none"):
        raise ValueError(f"unknown compression {compression}")
    if shard_inner is not None:
        chain = [{"name": "sharding_indexed", "configuration": {
            "chunk_shape": [int(c) for c in shard_inner], "codecs": chain,
            "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                             {"name": "crc32c"}],
            "index_location": "end"}}]
    return json.dumps(chain)


def create_array(path, data_type: str, shape, chunk_shape, codecs: Optional[str] = None,
                 fill_value=None) -> ArrayInfo:
    """ArrayBuilder::build + store_metadata for a filesystem store."""
    shape = [int(s) for s in shape]
    fv = None if fill_value is None else json.dumps(fill_value).encode()
    check(lib().zt_store_create_array(_b(path), _dt(data_type), len(shape), i64_array(shape),
                                      i64_array(chunk_shape),
                                      None if codecs is None else codecs.encode(), fv))
    return open_array(path)


def read_array(path, start=None, shape=None, nthreads: int = 0,
               out: Optional[np.ndarray] = None) -> np.ndarray:
    """Array::retrieve_array_subset_ndarray into a numpy array (bfloat16 as raw uint16); `out`:
    an existing C-contiguous array of that shape and type to fill (e.g. a view of pinned host
    memory)."""
    info = open_array(path)
    start = [0] * info.ndim if start is None else [int(s) for s in start]
    shape = list(info.shape) if shape is None else [int(s) for s in shape]
    if out is None:
        out = np.empty(shape, dtype=NUMPY[info.data_type])
    elif (list(out.shape) != shape or out.dtype != np.dtype(NUMPY[info.data_type])
          or not out.flags["C_CONTIGUOUS"]):
        raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS, "read_array: bad out array")
    check(lib().zt_store_read_subset(_b(path), i64_array(start), i64_array(shape),
                                     out.ctypes.data_as(ctypes.c_void_p), int(nthreads)))
    return out


def write_array(path, data: np.ndarray, start=None, nthreads: int = 0) -> None:
    """Array::store_array_subset_ndarray for a chunk-aligned subset."""
    info = open_array(path)
    data = np.ascontiguousarray(data)
    start = [0] * info.ndim if start is None else [int(s) for s in start]
    check(lib().zt_store_write_subset(_b(path), i64_array(start), i64_array(data.shape),
                                      data.ctypes.data_as(ctypes.c_void_p), int(nthreads)))


def write_synth(path, kind: int = SYNTH_STEP_NOISE_F32, seed: int = SEED,
                nthreads: int = 0) -> None:
    """Fill an array with the SURVEY.md §8(d) synthetic volume (same values as the device
    generator and oracle.synth_step_noise_f32 / synth_u16)."""
    check(lib().zt_store_write_synth(_b(path), int(kind), int(seed), int(nthreads)))


def codec_available(name: str) -> bool:
    return bool(lib().zt_store_codec_available(name.encode()))


def _enc(encoding) -> Optional[bytes]:
    """Reencoding arguments (ZarrReencodingArgs keys, lib.rs:274-377) as the ABI's JSON."""
    if encoding is None:
        return None
    if isinstance(encoding, (bytes, str)):
        return encoding.encode() if isinstance(encoding, str) else encoding
    return json.dumps({k: v for k, v in encoding.items() if v is not None}).encode()


_progress_keep = None


def set_progress_callback(fn) -> None:
    """Per-chunk progress of the store filters (Progress, progress.rs:15-119): `fn(stats)` with
    stats = {step, num_steps, read_s, process_s, write_s} after every output chunk is written.
    Process-wide; None disables."""
    global _progress_keep
    if fn is None:
        lib().zt_store_set_progress_callback(_abi.PROGRESS_FN(), None)
        _progress_keep = None
        return

    def _cb(p, _user):
        s = p.contents
        fn({"step": s.step, "num_steps": s.num_steps, "read_s": s.read_s,
            "process_s": s.process_s, "write_s": s.write_s})

    _progress_keep = _abi.PROGRESS_FN(_cb)
    lib().zt_store_set_progress_callback(_progress_keep, None)


def create_output_like(input_path, output_path, data_type: Optional[str] = None,
                       encoding=None) -> None:
    """The output array a filter creates (output_array_builder, filter_traits.rs:47-82), with
    its zarr.json written."""
    check(lib().zt_store_create_output_like(_b(input_path), _b(output_path), _dt(data_type),
                                            _enc(encoding)))


def create_output(input_path, output_path, data_type: Optional[str] = None, shape=None,
                  encoding=None) -> None:
    """The output array of a filter step with an explicit shape (None = the input's), as the
    store filters create it (reencoding included), zarr.json written, no chunk data."""
    nd = 0 if shape is None else len(shape)
    check(lib().zt_store_create_output(_b(input_path), _b(output_path), _dt(data_type),
                                       None if shape is None else i64_array(shape), nd,
                                       _enc(encoding)))


def host_available_bytes() -> int:
    """Host memory the store pipeline may budget (as host_available_bytes in host/zt_store.cpp):
    ZT_STORE_HOST_MEMORY if set, else MemAvailable capped at the cgroup's limit minus its usage,
    the usage without the cgroup's inactive file pages (reclaimable page cache, which MemAvailable
    counts as available). ZT_MEMINFO / ZT_CGROUP_ROOT relocate the files read (tests)."""
    env = os.environ.get("ZT_STORE_HOST_MEMORY")
    if env:
        return int(env)
    avail = 16 << 30
    try:
        with open(os.environ.get("ZT_MEMINFO", "/proc/meminfo")) as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    avail = int(line.split()[1]) * 1024
                    break
    except OSError:
        pass

    def _u64(path):
        try:
            with open(path) as f:
                t = f.read().strip()
            return int(t) if t.isdigit() else None
        except OSError:
            return None

    def _stat(path, key):
        try:
            with open(path) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == key:
                        return int(v)
        except (OSError, ValueError):
            pass
        return 0

    root = os.environ.get("ZT_CGROUP_ROOT", "/sys/fs/cgroup")
    for lim_p, use_p, stat_p, key in (
            ("memory.max", "memory.current", "memory.stat", "inactive_file"),
            ("memory/memory.limit_in_bytes", "memory/memory.usage_in_bytes",
             "memory/memory.stat", "total_inactive_file")):
        lim, use = _u64(os.path.join(root, lim_p)), _u64(os.path.join(root, use_p))
        if lim is not None and use is not None:
            if lim < (1 << 60):
                used = max(0, use - _stat(os.path.join(root, stat_p), key))
                avail = min(avail, max(0, lim - used))
            break
    return avail


PENDING_METADATA = ".zt_pending.json"  # kPendingMetadata, host/zt_zarr.hpp


def hold_metadata(path) -> None:
    """Hide a new array's zarr.json until its chunks are written ("not finished",
    zarrs_filter.rs:297-313; the reference stores metadata after the chunks): Zarr readers do not
    see the array, the store functions of this package still open it."""
    os.replace(os.path.join(path, "zarr.json"), os.path.join(path, PENDING_METADATA))


def publish_metadata(path) -> None:
    """The array is finished: its held metadata becomes zarr.json (an atomic rename)."""
    os.replace(os.path.join(path, PENDING_METADATA), os.path.join(path, "zarr.json"))


def set_chunk_limit(chunk_limit) -> None:
    """--chunk-limit for the store filters this thread calls next: at most that many chunks in
    flight (zt_store_set_chunk_limit; 0 / None = bounded by memory only)."""
    check(lib().zt_store_set_chunk_limit(int(chunk_limit or 0)))


def _flags(erase: bool, finish: bool) -> int:
    return (_abi.STORE_ERASE_OUTPUT_METADATA if erase else 0) | (
        _abi.STORE_FINISH_OUTPUT if finish else 0)


def guided_filter(input_path, output_path, epsilon: float, radius: int,
                  data_type: Optional[str] = None, device: int = 0, rows=None,
                  nthreads: int = 0, erase: bool = True, finish: bool = True,
                  encoding=None, chunk_limit: int = 0, cols=None) -> dict:
    """zarrs_filter guided-filter INPUT OUTPUT EPSILON RADIUS [--data-type T] on GPU `device`.
    `rows` = (begin, end) output chunk rows along axis 0 (None = all); `cols` = (begin, end)
    output chunk columns along axis 1 (None = all; a (t, z) block of a multi-GPU split);
    `chunk_limit` = at most that many chunks in flight (--chunk-limit, 0 = memory-bounded).
    Returns the run stats."""
    set_chunk_limit(chunk_limit)
    st = _abi.StoreStats()
    r0, r1 = (0, -1) if rows is None else (int(rows[0]), int(rows[1]))
    c0, c1 = (0, -1) if cols is None else (int(cols[0]), int(cols[1]))
    check(lib().zt_store_guided_filter_box(_b(input_path), _b(output_path), _dt(data_type),
                                           _enc(encoding), float(epsilon), int(radius),
                                           int(device), r0, r1, c0, c1, int(nthreads),
                                           _flags(erase, finish), ctypes.byref(st)))
    return st.as_dict()


def downsample(input_path, output_path, stride, discrete: bool = False,
               data_type: Optional[str] = None, device: int = 0, rows=None, nthreads: int = 0,
               erase: bool = True, finish: bool = True, encoding=None,
               chunk_limit: int = 0) -> dict:
    """zarrs_filter downsample INPUT OUTPUT STRIDE [--discrete] / one zarrs_ome level."""
    set_chunk_limit(chunk_limit)
    st = _abi.StoreStats()
    r0, r1 = (0, -1) if rows is None else (int(rows[0]), int(rows[1]))
    check(lib().zt_store_downsample(_b(input_path), _b(output_path), i64_array(stride),
                                    int(bool(discrete)), _dt(data_type), _enc(encoding),
                                    int(device), r0, r1,
                                    int(nthreads), _flags(erase, finish), ctypes.byref(st)))
    return st.as_dict()


def _sigma_half(sigma, kernel_half_size):
    sigma = [float(x) for x in sigma]
    half = [int(x) for x in kernel_half_size]
    return (ctypes.c_float * len(sigma))(*sigma), i64_array(half)


def gaussian(input_path, output_path, sigma, kernel_half_size, data_type: Optional[str] = None,
             device: int = 0, rows=None, nthreads: int = 0, erase: bool = True,
             finish: bool = True, encoding=None, chunk_limit: int = 0) -> dict:
    """zarrs_filter gaussian INPUT OUTPUT SIGMA KERNEL_HALF_SIZE [--data-type T]."""
    set_chunk_limit(chunk_limit)
    st = _abi.StoreStats()
    r0, r1 = (0, -1) if rows is None else (int(rows[0]), int(rows[1]))
    sg, hs = _sigma_half(sigma, kernel_half_size)
    check(lib().zt_store_gaussian(_b(input_path), _b(output_path), _dt(data_type),
                                  _enc(encoding), sg, hs,
                                  int(device), r0, r1, int(nthreads), _flags(erase, finish),
                                  ctypes.byref(st)))
    return st.as_dict()


def downsample_gaussian(input_path, output_path, stride, sigma, kernel_half_size,
                        data_type: Optional[str] = None, device: int = 0, rows=None,
                        nthreads: int = 0, erase: bool = True, finish: bool = True,
                        encoding=None, chunk_limit: int = 0) -> dict:
    """One zarrs_ome level with --gaussian-sigma (zarrs_ome.rs:236-271)."""
    set_chunk_limit(chunk_limit)
    st = _abi.StoreStats()
    r0, r1 = (0, -1) if rows is None else (int(rows[0]), int(rows[1]))
    sg, hs = _sigma_half(sigma, kernel_half_size)
    check(lib().zt_store_downsample_gaussian(_b(input_path), _b(output_path), i64_array(stride),
                                             sg, hs, _dt(data_type), _enc(encoding),
                                             int(device), r0, r1,
                                             int(nthreads), _flags(erase, finish),
                                             ctypes.byref(st)))
    return st.as_dict()
