"""Host-side mirror of the reference's filter-operator surface for the hot path.

Names, argument meaning and error behaviour follow LDeakin/zarrs_tools 0.7.2:
  - ``GuidedFilter`` <- src/filter/filters/guided_filter.rs (GuidedFilter::new(epsilon, radius,
    chunk_limit), apply_ndarray :117, apply_chunk :75, apply :240, is_compatible :203,
    memory_per_chunk :229)
  - ``Downsample`` <- src/filter/filters/downsample.rs (Downsample::new(stride, discrete,
    chunk_limit), input_subset :64, apply_ndarray_continuous :72, apply_ndarray_discrete :99,
    output_shape :162, apply :170)
  - ``ArraySubsetOverlap`` <- src/filter/array_subset_overlap.rs:4-52
Arrays are device-resident torch tensors (torch is used only for device memory and streams);
every computation runs in libzarrs_tools_amd.so through the C ABI.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import Optional, Sequence

from . import _abi
from ._abi import DTYPES, check, i64_array, lib


def _torch():
    import torch
    return torch


def torch_dtype(name: str):
    torch = _torch()
    return {
        "bool": torch.uint8, "int8": torch.int8, "int16": torch.int16, "int32": torch.int32,
        "int64": torch.int64, "uint8": torch.uint8, "uint16": torch.uint16,
        "uint32": torch.uint32, "uint64": torch.uint64, "bfloat16": torch.bfloat16,
        "float16": torch.float16, "float32": torch.float32, "float64": torch.float64,
    }[name]


def dtype_of(t) -> str:
    torch = _torch()
    m = {torch.int8: "int8", torch.int16: "int16", torch.int32: "int32", torch.int64: "int64",
         torch.uint8: "uint8", torch.uint16: "uint16", torch.uint32: "uint32",
         torch.uint64: "uint64", torch.bfloat16: "bfloat16", torch.float16: "float16",
         torch.float32: "float32", torch.float64: "float64", torch.bool: "bool"}
    return m[t.dtype]


class Context:
    """One HIP stream + scratch per (host thread, device) (zt_ctx)."""

    def __init__(self, device: int = 0, stream=None):
        h = ctypes.c_void_p()
        check(lib().zt_ctx_create(int(device), ctypes.byref(h)))
        self._h = h
        self.device = device
        if stream is not None:
            self.set_stream(stream)

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream) -> None:
        ptr = getattr(stream, "cuda_stream", stream)
        check(lib().zt_ctx_set_stream(self._h, ctypes.c_void_p(ptr)))

    def synchronize(self) -> None:
        check(lib().zt_ctx_synchronize(self._h))

    def scratch_bytes(self) -> int:
        n = ctypes.c_uint64()
        check(lib().zt_ctx_scratch_bytes(self._h, ctypes.byref(n)))
        return int(n.value)

    def release_scratch(self) -> None:
        """Free the device scratch the context keeps between calls."""
        check(lib().zt_ctx_release_scratch(self._h))

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_float()
        check(lib().zt_ctx_last_kernel_ms(self._h, ctypes.byref(ms)))
        return float(ms.value)

    def close(self) -> None:
        if self._h:
            lib().zt_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx: dict[int, Context] = {}


def default_context(device: Optional[int] = None) -> Context:
    torch = _torch()
    if device is None:
        device = torch.cuda.current_device()
    ctx = _default_ctx.get(device)
    if ctx is None:
        ctx = Context(device)
        _default_ctx[device] = ctx
    ctx.set_stream(torch.cuda.current_stream(device))
    return ctx


def _ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


@dataclass
class ArraySubset:
    start: tuple
    shape: tuple

    @property
    def end_exc(self):
        return tuple(s + n for s, n in zip(self.start, self.shape))


class ArraySubsetOverlap:
    """array_subset_overlap.rs:4-52 (computed by zt_subset_overlap)."""

    def __init__(self, shape_src: Sequence[int], subset_src: ArraySubset,
                 overlap: Sequence[int]):
        nd = len(shape_src)
        istart, ishape, dst = i64_array([0] * nd), i64_array([0] * nd), i64_array([0] * nd)
        check(lib().zt_subset_overlap(i64_array(shape_src), nd, i64_array(subset_src.start),
                                      i64_array(subset_src.shape), i64_array(overlap), istart,
                                      ishape, dst))
        self._input = ArraySubset(tuple(istart[:nd]), tuple(ishape[:nd]))
        self._dst = ArraySubset(tuple(dst[:nd]), tuple(subset_src.shape))

    def subset_input(self) -> ArraySubset:
        return self._input

    def subset_dst_in_src(self) -> ArraySubset:
        return self._dst

    def extract_subset(self, array):
        sl = tuple(slice(s, e) for s, e in zip(self._dst.start, self._dst.end_exc))
        return array[sl].clone()


class DeviceArray:
    """A device-resident chunked array: the in-HBM analogue of zarrs::Array for this path."""

    def __init__(self, data, chunk_shape: Sequence[int], dtype: Optional[str] = None):
        self.data = data
        self.chunk_shape = tuple(int(c) for c in chunk_shape)
        self.dtype = dtype or dtype_of(data)

    @property
    def shape(self):
        return tuple(self.data.shape)

    def chunk_grid_shape(self):
        return tuple(-(-s // c) for s, c in zip(self.shape, self.chunk_shape))

    def chunk_subset_bounded(self, chunk_indices) -> ArraySubset:
        start = tuple(i * c for i, c in zip(chunk_indices, self.chunk_shape))
        shape = tuple(min(s + c, n) - s for s, c, n in zip(start, self.chunk_shape, self.shape))
        return ArraySubset(start, shape)


def _check_radius(radius: int) -> int:
    r = int(radius)
    if not 0 <= r <= 255:
        raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS, "radius is a u8")
    return r


class GuidedFilter:
    """guided_filter.rs:52-320 — `GuidedFilter::new(epsilon, radius, chunk_limit)`."""

    def __init__(self, epsilon: float, radius: int, chunk_limit: Optional[int] = None):
        self._epsilon = float(epsilon)
        self._radius = _check_radius(radius)
        self.chunk_limit = chunk_limit

    def epsilon(self) -> float:
        return self._epsilon

    def radius(self) -> int:
        return self._radius

    def name(self) -> str:
        return "guided_filter"

    def is_compatible(self, dtype_in: str, dtype_out: str) -> None:
        for d in (dtype_in, dtype_out):
            if d not in DTYPES:
                raise _abi.UnsupportedDataType(_abi.ERR_UNSUPPORTED_DATA_TYPE,
                                               f"Unsupported data type {d}")
        check(lib().zt_guided_filter_is_compatible(DTYPES[dtype_in], DTYPES[dtype_out]))

    def memory_per_chunk(self, dtype_in: str, dtype_out: str, chunk_shape) -> int:
        out = ctypes.c_uint64()
        check(lib().zt_guided_filter_memory_per_chunk(DTYPES[dtype_in], DTYPES[dtype_out],
                                                      i64_array(chunk_shape), len(chunk_shape),
                                                      ctypes.byref(out)))
        return int(out.value)

    def apply_ndarray(self, v, out_subset: Optional[ArraySubset] = None,
                      dtype_out: Optional[str] = None, ctx: Optional[Context] = None):
        """guided_filter.rs:117-164 (+ extract_subset and the `as` casts of apply_chunk).

        `v` is the (halo'd) device block. Returns the filtered `out_subset` of the block
        (the whole block by default) as `dtype_out` (default: the input's dtype)."""
        torch = _torch()
        ctx = ctx or default_context(v.device.index)
        dtype_in = dtype_of(v)
        dtype_out = dtype_out or dtype_in
        nd = v.dim()
        if out_subset is None:
            out_subset = ArraySubset((0,) * nd, tuple(v.shape))
        out = torch.empty(out_subset.shape, dtype=torch_dtype(dtype_out), device=v.device)
        in_strides = i64_array(v.stride())
        check(lib().zt_guided_filter_apply_ndarray(
            ctx.handle, DTYPES[dtype_in], _ptr(v), i64_array(v.shape), in_strides, nd,
            i64_array(out_subset.start), i64_array(out_subset.shape), DTYPES[dtype_out], _ptr(out),
            i64_array(out.stride()), self._epsilon, self._radius))
        return out

    def apply_chunk(self, input: DeviceArray, output: DeviceArray, chunk_indices,
                    ctx: Optional[Context] = None) -> None:
        """guided_filter.rs:75-114 on device-resident arrays: halo'd read, filter, interior
        write."""
        subset_output = output.chunk_subset_bounded(chunk_indices)
        overlap = ArraySubsetOverlap(input.shape, subset_output,
                                     [(self._radius * 2) & 0xFF] * len(input.shape))
        si = overlap.subset_input()
        block = input.data[tuple(slice(s, s + n) for s, n in zip(si.start, si.shape))]
        res = self.apply_ndarray(block, overlap.subset_dst_in_src(), output.dtype, ctx)
        output.data[tuple(slice(s, s + n) for s, n in
                          zip(subset_output.start, subset_output.shape))] = res

    def apply(self, input: DeviceArray, output: DeviceArray, ctx: Optional[Context] = None,
              chunk_grid_start=None, chunk_grid_count=None) -> None:
        """guided_filter.rs:240-319 over every output chunk (batched into one launch)."""
        if tuple(output.shape) != tuple(input.shape):
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         "input and output shapes differ")
        ctx = ctx or default_context(input.data.device.index)
        nd = len(input.shape)
        check(lib().zt_guided_filter_apply_array(
            ctx.handle, DTYPES[input.dtype], _ptr(input.data), DTYPES[output.dtype],
            _ptr(output.data), i64_array(input.shape), nd, i64_array(output.chunk_shape),
            self._epsilon, self._radius,
            None if chunk_grid_start is None else i64_array(chunk_grid_start),
            None if chunk_grid_count is None else i64_array(chunk_grid_count)))


class Gaussian:
    """gaussian.rs:49-250 — `Gaussian::new(sigma, kernel_half_size, chunk_limit)`: the separable
    sampled Gaussian, per axis in order, replicate edges (kernel.rs:17-73)."""

    def __init__(self, sigma: Sequence[float], kernel_half_size: Sequence[int],
                 chunk_limit: Optional[int] = None):
        self.sigma = tuple(float(s) for s in sigma)
        self._half = tuple(int(h) for h in kernel_half_size)
        if len(self.sigma) != len(self._half):
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         "sigma and kernel_half_size lengths differ")
        self.chunk_limit = chunk_limit

    def name(self) -> str:
        return "gaussian"

    def kernel_half_size(self) -> tuple:
        return self._half

    def kernel(self, axis: int) -> list:
        """create_sampled_gaussian_kernel (gaussian.rs:252-267) for one axis."""
        n = ctypes.c_int64()
        check(lib().zt_gaussian_kernel(self.sigma[axis], self._half[axis], None, ctypes.byref(n)))
        taps = (ctypes.c_float * n.value)()
        check(lib().zt_gaussian_kernel(self.sigma[axis], self._half[axis], taps, ctypes.byref(n)))
        return list(taps)

    def _args(self, nd: int):
        if len(self.sigma) != nd:
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         "sigma / kernel_half_size must have one entry per axis")
        return (ctypes.c_float * nd)(*self.sigma), i64_array(self._half)

    def is_compatible(self, dtype_in: str, dtype_out: str) -> None:
        for d in (dtype_in, dtype_out):
            if d not in DTYPES:
                raise _abi.UnsupportedDataType(_abi.ERR_UNSUPPORTED_DATA_TYPE,
                                               f"Unsupported data type {d}")
        check(lib().zt_gaussian_is_compatible(DTYPES[dtype_in], DTYPES[dtype_out]))

    def memory_per_chunk(self, dtype_in: str, dtype_out: str, chunk_shape) -> int:
        out = ctypes.c_uint64()
        check(lib().zt_gaussian_memory_per_chunk(DTYPES[dtype_in], DTYPES[dtype_out],
                                                 i64_array(chunk_shape), len(chunk_shape),
                                                 i64_array(self._half), ctypes.byref(out)))
        return int(out.value)

    def apply_ndarray(self, v, out_subset: Optional[ArraySubset] = None,
                      dtype_out: Optional[str] = None, ctx: Optional[Context] = None):
        """gaussian.rs:110-119 (+ extract_subset and the `as` casts of apply_chunk) on a
        device block; returns `out_subset` of the result (whole block by default)."""
        torch = _torch()
        v = v.contiguous()
        ctx = ctx or default_context(v.device.index)
        dtype_in = dtype_of(v)
        dtype_out = dtype_out or dtype_in
        nd = v.dim()
        if out_subset is None:
            out_subset = ArraySubset((0,) * nd, tuple(v.shape))
        sig, half = self._args(nd)
        out = torch.empty(out_subset.shape, dtype=torch_dtype(dtype_out), device=v.device)
        check(lib().zt_gaussian_apply_ndarray(
            ctx.handle, DTYPES[dtype_in], _ptr(v), i64_array(v.shape), nd,
            i64_array(out_subset.start), i64_array(out_subset.shape), DTYPES[dtype_out],
            _ptr(out), sig, half))
        return out

    def apply_chunk(self, input: DeviceArray, output: DeviceArray, chunk_indices,
                    ctx: Optional[Context] = None) -> None:
        """gaussian.rs:73-108 on device-resident arrays."""
        subset_output = output.chunk_subset_bounded(chunk_indices)
        overlap = ArraySubsetOverlap(input.shape, subset_output, self._half)
        si = overlap.subset_input()
        block = input.data[tuple(slice(s, s + n) for s, n in zip(si.start, si.shape))]
        res = self.apply_ndarray(block, overlap.subset_dst_in_src(), output.dtype, ctx)
        output.data[tuple(slice(s, s + n) for s, n in
                          zip(subset_output.start, subset_output.shape))] = res

    def apply(self, input: DeviceArray, output: DeviceArray,
              ctx: Optional[Context] = None) -> None:
        """gaussian.rs:170-249 over every output chunk (one pass over the array)."""
        if tuple(output.shape) != tuple(input.shape):
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         "input and output shapes differ")
        ctx = ctx or default_context(input.data.device.index)
        nd = len(input.shape)
        sig, half = self._args(nd)
        check(lib().zt_gaussian_apply_array(
            ctx.handle, DTYPES[input.dtype], _ptr(input.data.contiguous()), DTYPES[output.dtype],
            _ptr(output.data), i64_array(input.shape), nd, i64_array(output.chunk_shape), sig,
            half))


class Downsample:
    """downsample.rs:49-287 — `Downsample::new(stride, discrete, chunk_limit)`."""

    def __init__(self, stride: Sequence[int], discrete: bool = False,
                 chunk_limit: Optional[int] = None):
        self.stride = tuple(int(s) for s in stride)
        self.discrete = bool(discrete)
        self.chunk_limit = chunk_limit

    def name(self) -> str:
        return "downsample"

    def is_compatible(self, dtype_in: str, dtype_out: str) -> None:
        check(lib().zt_downsample_is_compatible(DTYPES[dtype_in], DTYPES[dtype_out],
                                                int(self.discrete)))

    def output_shape(self, input_shape) -> tuple:
        nd = len(input_shape)
        out = i64_array([0] * nd)
        check(lib().zt_downsample_output_shape(i64_array(input_shape), nd,
                                               i64_array(self.stride), out))
        return tuple(out[:nd])

    def input_subset(self, input_shape, output_subset: ArraySubset) -> ArraySubset:
        nd = len(input_shape)
        s, n = i64_array([0] * nd), i64_array([0] * nd)
        check(lib().zt_downsample_input_subset(i64_array(input_shape), nd, i64_array(self.stride),
                                               i64_array(output_subset.start),
                                               i64_array(output_subset.shape), s, n))
        return ArraySubset(tuple(s[:nd]), tuple(n[:nd]))

    def _apply(self, v, dtype_out, discrete, ctx):
        torch = _torch()
        v = v.contiguous()
        ctx = ctx or default_context(v.device.index)
        dtype_in = dtype_of(v)
        dtype_out = dtype_out or dtype_in
        nd = v.dim()
        win = [min(s, n) for s, n in zip(self.stride, v.shape)]
        oshape = [n // w if w > 0 else 0 for n, w in zip(v.shape, win)]
        out = torch.empty(oshape, dtype=torch_dtype(dtype_out), device=v.device)
        check(lib().zt_downsample_apply_ndarray(ctx.handle, DTYPES[dtype_in], _ptr(v),
                                                i64_array(v.shape), nd, i64_array(self.stride),
                                                int(discrete), DTYPES[dtype_out], _ptr(out)))
        return out

    def apply_ndarray_continuous(self, v, dtype_out: Optional[str] = None,
                                 ctx: Optional[Context] = None):
        """downsample.rs:72-97"""
        return self._apply(v, dtype_out, False, ctx)

    def apply_ndarray_discrete(self, v, dtype_out: Optional[str] = None,
                               ctx: Optional[Context] = None):
        """downsample.rs:99-120 (ties -> smallest value)"""
        return self._apply(v, dtype_out, True, ctx)

    def apply(self, input: DeviceArray, output: DeviceArray, ctx: Optional[Context] = None):
        """downsample.rs:170-286: the whole output array (chunk-independent, one launch)."""
        if tuple(output.shape) != self.output_shape(input.shape):
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS, "output shape mismatch")
        # Per chunk the reference reads input_subset(output chunk) and keeps complete windows;
        # with out = max(shape/stride, 1) those are exactly the whole-array windows.
        res = self._apply(input.data, output.dtype, self.discrete, ctx)
        output.data.copy_(res.reshape(output.data.shape))


def reencode_cast(v, dtype_out: str, ctx: Optional[Context] = None):
    """Reencode::apply_chunk_convert's element conversion (reencode.rs:58-77) on a device tensor:
    every element `as` dtype_out (zt_reencode_cast). Returns a new contiguous tensor; bfloat16 is
    torch.bfloat16."""
    torch = _torch()
    v = v.contiguous()
    ctx = ctx or default_context(v.device.index)
    dtype_in = dtype_of(v)
    out = torch.empty(tuple(v.shape), dtype=torch_dtype(dtype_out), device=v.device)
    check(lib().zt_reencode_cast(ctx.handle, DTYPES[dtype_in], _ptr(v), DTYPES[dtype_out],
                                 _ptr(out), int(v.numel())))
    return out


def pyramid_level_shapes(shape, factor, max_levels: int) -> list:
    """zarrs_ome.rs:515-560/:731-737 level shapes + stop rule."""
    nd = len(shape)
    buf = i64_array([0] * (nd * max(max_levels, 1)))
    n = ctypes.c_int()
    check(lib().zt_pyramid_level_shapes(i64_array(shape), nd, i64_array(factor), int(max_levels),
                                        buf, ctypes.byref(n)))
    return [tuple(buf[i * nd:(i + 1) * nd]) for i in range(n.value)]


def pyramid(level0, factor=None, max_levels: int = 10, discrete: bool = False,
            ctx: Optional[Context] = None) -> list:
    """Device-resident zarrs_ome mean (or mode) pyramid: returns [level1, level2, ...]."""
    torch = _torch()
    level0 = level0.contiguous()
    ctx = ctx or default_context(level0.device.index)
    nd = level0.dim()
    factor = tuple(factor or (2,) * nd)
    shapes = pyramid_level_shapes(level0.shape, factor, max_levels)
    outs = [torch.empty(s, dtype=level0.dtype, device=level0.device) for s in shapes]
    ptrs = (ctypes.c_void_p * max(len(outs), 1))(*[o.data_ptr() for o in outs])
    written = ctypes.c_int()
    check(lib().zt_pyramid_downsample(ctx.handle, DTYPES[dtype_of(level0)], _ptr(level0),
                                      i64_array(level0.shape), nd, i64_array(factor),
                                      int(max_levels), int(discrete), ptrs, ctypes.byref(written)))
    return outs[:written.value]


def synth_step_noise_f32(shape, seed: int = 0x5EED2025, global_shape=None, z0: int = 0,
                         device=None, ctx: Optional[Context] = None):
    """SURVEY.md §8(d) synthetic volume generated on the device."""
    torch = _torch()
    out = torch.empty(tuple(shape), dtype=torch.float32, device=device or "cuda")
    ctx = ctx or default_context(out.device.index)
    gs = global_shape or shape
    check(lib().zt_synth_step_noise_f32(ctx.handle, _ptr(out), i64_array(shape), len(shape),
                                        i64_array(gs), int(z0), int(seed)))
    return out


def synth_u16(shape, seed: int = 0x5EED2025, global_shape=None, z0: int = 0, device=None,
              ctx: Optional[Context] = None):
    torch = _torch()
    out = torch.empty(tuple(shape), dtype=torch.uint16, device=device or "cuda")
    ctx = ctx or default_context(out.device.index)
    gs = global_shape or shape
    check(lib().zt_synth_u16(ctx.handle, _ptr(out), i64_array(shape), len(shape), i64_array(gs),
                             int(z0), int(seed)))
    return out


def synth_box(start, shape, global_shape, kind: str = "uint16", seed: int = 0x5EED2025,
              device=None, ctx: Optional[Context] = None):
    """The box [start, start+shape) of the global synthetic volume, generated on the device
    (kind "uint16" noise or "float32" step+noise): a rank's own octant or slab."""
    torch = _torch()
    dt = torch.uint16 if kind == "uint16" else torch.float32
    out = torch.empty(tuple(shape), dtype=dt, device=device or "cuda")
    ctx = ctx or default_context(out.device.index)
    check(lib().zt_synth_box(ctx.handle, 1 if kind == "uint16" else 0, _ptr(out),
                             i64_array(start), i64_array(shape), i64_array(global_shape),
                             len(shape), int(seed)))
    return out
