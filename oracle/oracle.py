"""ctypes binding of the C oracle (oracle/zt_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker / the timed CPU baseline. The product package (zarrs_tools_amd) never imports it.
The functions mirror the reference restatement cited in oracle/zt_oracle.h.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libzt_oracle.so")
_lib = None

# dtype codes shared with include/zarrs_tools_amd.h
DTYPES = {
    "bool": 0, "int8": 1, "int16": 2, "int32": 3, "int64": 4,
    "uint8": 5, "uint16": 6, "uint32": 7, "uint64": 8,
    "bfloat16": 9, "float16": 10, "float32": 11, "float64": 12,
}
# numpy storage type of each element type (bf16 stored as raw uint16 bits)
NP_STORAGE = {
    "bool": np.uint8, "int8": np.int8, "int16": np.int16, "int32": np.int32, "int64": np.int64,
    "uint8": np.uint8, "uint16": np.uint16, "uint32": np.uint32, "uint64": np.uint64,
    "bfloat16": np.uint16, "float16": np.uint16, "float32": np.float32, "float64": np.float64,
}

SEED = 0x5EED2025


def build() -> str:
    """Compile the oracle with its Makefile (gcc); returns the library path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i64p = ctypes.POINTER(ctypes.c_int64)
        vp = ctypes.c_void_p
        L.oracle_summed_area_table.argtypes = [vp, vp, i64p, ctypes.c_int]
        L.oracle_guided_filter_apply_ndarray.argtypes = [vp, i64p, ctypes.c_int, ctypes.c_float,
                                                         ctypes.c_int, ctypes.c_int]
        L.oracle_guided_filter_apply.argtypes = [vp, vp, i64p, ctypes.c_int, i64p, ctypes.c_float,
                                                 ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_guided_filter_apply.restype = ctypes.c_int
        L.oracle_guided_filter_apply_chunks.argtypes = [
            vp, vp, i64p, ctypes.c_int, i64p, ctypes.c_float, ctypes.c_int, ctypes.c_int,
            ctypes.c_int, ctypes.c_int64, ctypes.c_int64]
        L.oracle_guided_filter_apply_chunks.restype = ctypes.c_int64
        for name in ("oracle_cast_from_f32", "oracle_cast_from_f64"):
            getattr(L, name).argtypes = [vp, ctypes.c_int, vp, ctypes.c_int64]
        for name in ("oracle_cast_to_f32", "oracle_cast_to_f64"):
            getattr(L, name).argtypes = [vp, ctypes.c_int, vp, ctypes.c_int64]
        for name in ("oracle_downsample_continuous", "oracle_downsample_discrete"):
            f = getattr(L, name)
            f.argtypes = [vp, ctypes.c_int, i64p, ctypes.c_int, i64p, vp, ctypes.c_int]
            f.restype = ctypes.c_int
        L.oracle_splitmix64.argtypes = [ctypes.c_uint64]
        L.oracle_splitmix64.restype = ctypes.c_uint64
        L.oracle_synth_step_noise_f32.argtypes = [vp, i64p, ctypes.c_int, i64p, ctypes.c_int64,
                                                  ctypes.c_uint64]
        L.oracle_synth_u16.argtypes = [vp, i64p, ctypes.c_int, i64p, ctypes.c_int64,
                                       ctypes.c_uint64]
        L.oracle_synth_block_f32.argtypes = [vp, i64p, i64p, i64p, ctypes.c_uint64]
        for name in ("oracle_synth_block_nd_f32", "oracle_synth_block_nd_u16"):
            getattr(L, name).argtypes = [vp, i64p, i64p, i64p, ctypes.c_int, ctypes.c_uint64]
        L.oracle_guided_filter_time_chunks.argtypes = [
            i64p, i64p, i64p, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int,
            ctypes.c_uint64, i64p]
        L.oracle_guided_filter_time_chunks.restype = ctypes.c_double
        fp = ctypes.POINTER(ctypes.c_float)
        L.oracle_gaussian_kernel.argtypes = [ctypes.c_float, ctypes.c_int64, fp]
        L.oracle_gaussian_kernel.restype = ctypes.c_int64
        L.oracle_gaussian_apply_ndarray.argtypes = [vp, i64p, ctypes.c_int, fp, i64p]
        L.oracle_gaussian_apply_ndarray.restype = ctypes.c_int
        L.oracle_gaussian_apply.argtypes = [vp, vp, i64p, ctypes.c_int, i64p, fp, i64p]
        L.oracle_gaussian_apply.restype = ctypes.c_int
        _lib = L
    return _lib


def _shape(shape):
    arr = (ctypes.c_int64 * len(shape))(*[int(s) for s in shape])
    return arr


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def summed_area_table(v: np.ndarray) -> np.ndarray:
    v = np.ascontiguousarray(v, dtype=np.float32)
    sat = np.empty(v.shape, dtype=np.float64)
    lib().oracle_summed_area_table(_ptr(v), _ptr(sat), _shape(v.shape), v.ndim)
    return sat


def guided_filter_apply_ndarray(v: np.ndarray, epsilon: float, radius: int,
                                faithful: bool = False) -> np.ndarray:
    """GuidedFilter::apply_ndarray (guided_filter.rs:117-164) on one whole block."""
    out = np.array(v, dtype=np.float32, order="C", copy=True)
    lib().oracle_guided_filter_apply_ndarray(_ptr(out), _shape(out.shape), out.ndim,
                                             float(epsilon), int(radius), int(faithful))
    return out


def guided_filter_apply(v: np.ndarray, chunk_shape, epsilon: float, radius: int,
                        nthreads: int = 1, faithful: bool = False) -> np.ndarray:
    """GuidedFilter::apply (guided_filter.rs:240-319): chunked, 2r halo per output chunk."""
    v = np.ascontiguousarray(v, dtype=np.float32)
    out = np.empty_like(v)
    rc = lib().oracle_guided_filter_apply(_ptr(v), _ptr(out), _shape(v.shape), v.ndim,
                                          _shape(chunk_shape), float(epsilon), int(radius),
                                          int(nthreads), int(faithful))
    if rc != 0:
        raise ValueError(f"oracle_guided_filter_apply failed: {rc}")
    return out


def guided_filter_apply_chunks(v: np.ndarray, out: np.ndarray, chunk_shape, epsilon: float,
                               radius: int, nthreads: int, chunk_begin: int, chunk_end: int,
                               faithful: bool = True) -> int:
    return lib().oracle_guided_filter_apply_chunks(
        _ptr(v), _ptr(out), _shape(v.shape), v.ndim, _shape(chunk_shape), float(epsilon),
        int(radius), int(nthreads), int(faithful), int(chunk_begin), int(chunk_end))


def _floats(xs):
    return (ctypes.c_float * len(xs))(*[float(x) for x in xs])


def gaussian_kernel(sigma: float, half: int) -> np.ndarray:
    """create_sampled_gaussian_kernel (gaussian.rs:252-267)."""
    taps = (ctypes.c_float * (2 * int(half) + 1))()
    n = lib().oracle_gaussian_kernel(float(sigma), int(half), taps)
    return np.array(taps[:n], dtype=np.float32)


def gaussian_apply_ndarray(v: np.ndarray, sigma, kernel_half_size) -> np.ndarray:
    """Gaussian::apply_ndarray (gaussian.rs:110-119) on one whole block."""
    out = np.array(v, dtype=np.float32, order="C", copy=True)
    rc = lib().oracle_gaussian_apply_ndarray(_ptr(out), _shape(out.shape), out.ndim,
                                             _floats(sigma), _shape(kernel_half_size))
    if rc != 0:
        raise ValueError(f"oracle_gaussian_apply_ndarray failed: {rc}")
    return out


def gaussian_apply(v: np.ndarray, chunk_shape, sigma, kernel_half_size) -> np.ndarray:
    """Gaussian::apply (gaussian.rs:170-249): chunked, kernel_half_size halo per chunk."""
    v = np.ascontiguousarray(v, dtype=np.float32)
    out = np.empty_like(v)
    rc = lib().oracle_gaussian_apply(_ptr(v), _ptr(out), _shape(v.shape), v.ndim,
                                     _shape(chunk_shape), _floats(sigma),
                                     _shape(kernel_half_size))
    if rc != 0:
        raise ValueError(f"oracle_gaussian_apply failed: {rc}")
    return out


def cast_from_f32(v: np.ndarray, dtype: str) -> np.ndarray:
    v = np.ascontiguousarray(v, dtype=np.float32)
    out = np.empty(v.shape, dtype=NP_STORAGE[dtype])
    lib().oracle_cast_from_f32(_ptr(v), DTYPES[dtype], _ptr(out), v.size)
    return out


def cast_from_f64(v: np.ndarray, dtype: str) -> np.ndarray:
    v = np.ascontiguousarray(v, dtype=np.float64)
    out = np.empty(v.shape, dtype=NP_STORAGE[dtype])
    lib().oracle_cast_from_f64(_ptr(v), DTYPES[dtype], _ptr(out), v.size)
    return out


def cast_to_f32(v: np.ndarray, dtype: str) -> np.ndarray:
    v = np.ascontiguousarray(v, dtype=NP_STORAGE[dtype])
    out = np.empty(v.shape, dtype=np.float32)
    lib().oracle_cast_to_f32(_ptr(v), DTYPES[dtype], _ptr(out), v.size)
    return out


def downsample_output_shape(in_shape, stride):
    return tuple((s // min(st, s)) if s > 0 else 0 for s, st in zip(in_shape, stride))


def downsample(v: np.ndarray, dtype_in: str, stride, dtype_out: str,
               discrete: bool = False) -> np.ndarray:
    """Downsample::apply_ndarray_{continuous,discrete} (downsample.rs:72-120)."""
    v = np.ascontiguousarray(v, dtype=NP_STORAGE[dtype_in])
    oshape = downsample_output_shape(v.shape, stride)
    out = np.empty(oshape, dtype=NP_STORAGE[dtype_out])
    fn = lib().oracle_downsample_discrete if discrete else lib().oracle_downsample_continuous
    rc = fn(_ptr(v), DTYPES[dtype_in], _shape(v.shape), v.ndim, _shape(stride), _ptr(out),
            DTYPES[dtype_out])
    if rc != 0:
        raise ValueError(f"oracle downsample failed: {rc}")
    return out


def synth_step_noise_f32(shape, seed: int = SEED, global_shape=None, z0: int = 0) -> np.ndarray:
    """v = 500*[x >= nx/2] + 100*U(splitmix64(seed ^ index))."""
    shape = tuple(int(s) for s in shape)
    out = np.empty(shape, dtype=np.float32)
    gs = shape if global_shape is None else tuple(global_shape)
    lib().oracle_synth_step_noise_f32(_ptr(out), _shape(shape), len(shape), _shape(gs), int(z0),
                                      int(seed))
    return out


def synth_u16(shape, seed: int = SEED, global_shape=None, z0: int = 0) -> np.ndarray:
    shape = tuple(int(s) for s in shape)
    out = np.empty(shape, dtype=np.uint16)
    gs = shape if global_shape is None else tuple(global_shape)
    lib().oracle_synth_u16(_ptr(out), _shape(shape), len(shape), _shape(gs), int(z0), int(seed))
    return out


def synth_block_f32(start, shape, global_shape, seed: int = SEED) -> np.ndarray:
    out = np.empty(tuple(int(s) for s in shape), dtype=np.float32)
    lib().oracle_synth_block_f32(_ptr(out), _shape(start), _shape(shape), _shape(global_shape),
                                 int(seed))
    return out


def synth_block_nd(start, shape, global_shape, kind: str = "float32", seed: int = SEED
                   ) -> np.ndarray:
    """The box [start, start+shape) of the N-d global synthetic volume (step+noise f32 or u16
    noise), equal to the same box of synth_step_noise_f32 / synth_u16 over the whole array."""
    shape = tuple(int(s) for s in shape)
    if kind == "float32":
        out = np.empty(shape, dtype=np.float32)
        fn = lib().oracle_synth_block_nd_f32
    else:
        out = np.empty(shape, dtype=np.uint16)
        fn = lib().oracle_synth_block_nd_u16
    fn(_ptr(out), _shape(start), _shape(shape), _shape(global_shape), len(shape), int(seed))
    return out


def chunk_halo_subset(global_shape, chunk_shape, coord, halo):
    """chunk_subset_bounded + ArraySubsetOverlap::new (guided_filter.rs:87-93,
    array_subset_overlap.rs:11-35): (output start, output shape, input start, input shape)."""
    o0 = [c * s for c, s in zip(coord, chunk_shape)]
    o1 = [min(a + s, g) for a, s, g in zip(o0, chunk_shape, global_shape)]
    i0 = [max(a - halo, 0) for a in o0]
    i1 = [min(b + halo, g) for b, g in zip(o1, global_shape)]
    return (o0, [b - a for a, b in zip(o0, o1)], i0, [b - a for a, b in zip(i0, i1)])


def guided_filter_synth_chunks(global_shape, chunk_shape, coords, epsilon: float, radius: int,
                               nthreads: int = 8, seed: int = SEED):
    """Expected output of each listed chunk of the synthetic step+noise volume, computed the
    reference's way (GuidedFilter::apply_chunk, guided_filter.rs:75-114): the 2r-halo input
    subset clamped to the array, apply_ndarray on it, the halo dropped. Chunks run in parallel
    threads (ctypes releases the GIL). Returns [(out_start, out_shape, block)]."""
    from concurrent.futures import ThreadPoolExecutor
    halo = (2 * int(radius)) & 0xFF

    def one(coord):
        o0, osh, i0, ish = chunk_halo_subset(global_shape, chunk_shape, coord, halo)
        blk = synth_block_nd(i0, ish, global_shape, "float32", seed)
        res = guided_filter_apply_ndarray(blk, epsilon, radius)
        sl = tuple(slice(a - b, a - b + s) for a, b, s in zip(o0, i0, osh))
        return (o0, osh, np.ascontiguousarray(res[sl]))

    with ThreadPoolExecutor(max_workers=max(1, nthreads)) as ex:
        return list(ex.map(one, [tuple(c) for c in coords]))


def sample_chunk_coords(grid, n_interior: int = 2):
    """Corner, edge and interior chunks of a chunk grid: the first and last chunk, one with a
    single axis at its edge, and n_interior interior chunks (deduplicated)."""
    nd = len(grid)
    cs = [tuple(0 for _ in grid), tuple(g - 1 for g in grid)]
    cs.append(tuple(g // 2 if d else 0 for d, g in enumerate(grid)))           # face chunk
    cs.append(tuple(g - 1 if d == nd - 1 else g // 2 for d, g in enumerate(grid)))  # x edge
    for k in range(n_interior):
        cs.append(tuple(min(max(1, (g * (k + 1)) // (n_interior + 1)), max(g - 2, 0))
                        for g in grid))
    out = []
    for c in cs:
        if c not in out:
            out.append(c)
    return out


def time_guided_filter_chunks(global_shape, chunk_shape, chunk_coords, epsilon: float,
                              radius: int, nthreads: int, seed: int = SEED):
    """bench.py cpu_baseline: wall seconds of the reference algorithm on the listed chunks."""
    flat = [int(c) for cc in chunk_coords for c in cc]
    vox = ctypes.c_int64()
    secs = lib().oracle_guided_filter_time_chunks(
        _shape(global_shape), _shape(chunk_shape), _shape(flat), len(chunk_coords),
        float(epsilon), int(radius), int(nthreads), int(seed), ctypes.byref(vox))
    return float(secs), int(vox.value)
