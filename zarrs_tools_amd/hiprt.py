"""Minimal HIP runtime calls through ctypes, for processes that never import torch.

The octant workers of `zarrs_ome --gpus N` only move a box of level 0 into HBM, run the
level-fused pyramid (zt_pyramid_downsample) and copy the levels back: device and pinned host
allocations, copies on a stream and events are all they need. Without torch a spawned worker
starts in a fraction of a second instead of ~2 s (the torch import and its runtime set-up).

Such a process sets ZT_NO_TORCH=1 before importing this package, so `_abi.lib()` does not load
torch's HIP runtime first; the product library then binds the ROCm runtime of its RUNPATH, and
this module uses that same loaded copy (same soname). Not for processes that use torch.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _abi

_hip = None
H2D, D2H = 1, 2  # hipMemcpyKind


def hip() -> ctypes.CDLL:
    global _hip
    if _hip is None:
        _abi.lib()  # loads libamdhip64.so.7 as the product library's dependency
        L = ctypes.CDLL("libamdhip64.so.7")
        vp, c_int, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        sig = {
            "hipSetDevice": ([c_int], c_int),
            "hipMalloc": ([ctypes.POINTER(vp), sz], c_int),
            "hipFree": ([vp], c_int),
            "hipHostMalloc": ([ctypes.POINTER(vp), sz, ctypes.c_uint], c_int),
            "hipHostFree": ([vp], c_int),
            "hipMemcpyAsync": ([vp, vp, sz, c_int, vp], c_int),
            "hipMemcpy2DAsync": ([vp, sz, vp, sz, sz, sz, c_int, vp], c_int),
            "hipStreamCreate": ([ctypes.POINTER(vp)], c_int),
            "hipStreamDestroy": ([vp], c_int),
            "hipStreamSynchronize": ([vp], c_int),
            "hipEventCreate": ([ctypes.POINTER(vp)], c_int),
            "hipEventDestroy": ([vp], c_int),
            "hipEventRecord": ([vp, vp], c_int),
            "hipEventSynchronize": ([vp], c_int),
            "hipGetErrorString": ([c_int], ctypes.c_char_p),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        _hip = L
    return _hip


def check(err: int, what: str) -> None:
    if err != 0:
        msg = hip().hipGetErrorString(err).decode(errors="replace")
        raise _abi.FilterError(_abi.ERR_DEVICE, f"{what}: {msg}")


def set_device(device: int) -> None:
    check(hip().hipSetDevice(int(device)), "hipSetDevice")
    check(hip().hipFree(None), "device context")  # create the context now


class DeviceBuffer:
    """hipMalloc'd device memory (freed by free() or when collected)."""

    def __init__(self, nbytes: int):
        self.ptr = ctypes.c_void_p()
        self.nbytes = int(nbytes)
        check(hip().hipMalloc(ctypes.byref(self.ptr), max(self.nbytes, 1)), "hipMalloc")

    def at(self, offset: int) -> ctypes.c_void_p:
        return ctypes.c_void_p((self.ptr.value or 0) + int(offset))

    def free(self) -> None:
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:  # interpreter shutdown
            pass


NON_COHERENT = 0x80000000  # hipHostMallocNonCoherent


class PinnedBuffer:
    """hipHostMalloc'd (page-locked) host memory, viewed as numpy arrays. `flags`: the
    hipHostMalloc flags (NON_COHERENT suits buffers only stream-ordered copies touch on the
    device side; it falls back to the default when the runtime refuses it)."""

    def __init__(self, nbytes: int, flags: int = 0):
        self.ptr = ctypes.c_void_p()
        self.nbytes = int(nbytes)
        err = hip().hipHostMalloc(ctypes.byref(self.ptr), max(self.nbytes, 1), flags)
        if err != 0 and flags != 0:  # a runtime without the flag: the default pinned memory
            err = hip().hipHostMalloc(ctypes.byref(self.ptr), max(self.nbytes, 1), 0)
        check(err, "hipHostMalloc")

    def array(self, dtype, shape) -> np.ndarray:
        n = int(np.prod(shape)) * np.dtype(dtype).itemsize
        assert n <= self.nbytes
        raw = (ctypes.c_char * max(n, 1)).from_address(self.ptr.value)
        return np.frombuffer(raw, dtype=dtype, count=int(np.prod(shape))).reshape(shape)

    def free(self) -> None:
        if self.ptr:
            hip().hipHostFree(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:  # interpreter shutdown
            pass


class Stream:
    def __init__(self):
        self.handle = ctypes.c_void_p()
        check(hip().hipStreamCreate(ctypes.byref(self.handle)), "hipStreamCreate")

    def synchronize(self) -> None:
        check(hip().hipStreamSynchronize(self.handle), "hipStreamSynchronize")

    def __del__(self):
        try:
            if self.handle:
                hip().hipStreamDestroy(self.handle)
        except Exception:  # interpreter shutdown
            pass


class Event:
    def __init__(self):
        self.handle = ctypes.c_void_p()
        check(hip().hipEventCreate(ctypes.byref(self.handle)), "hipEventCreate")

    def record(self, stream: Stream) -> None:
        check(hip().hipEventRecord(self.handle, stream.handle), "hipEventRecord")

    def synchronize(self) -> None:
        check(hip().hipEventSynchronize(self.handle), "hipEventSynchronize")

    def __del__(self):
        try:
            if self.handle:
                hip().hipEventDestroy(self.handle)
        except Exception:  # interpreter shutdown
            pass


def copy_async(dst, src, nbytes: int, kind: int, stream: Stream) -> None:
    check(hip().hipMemcpyAsync(dst, src, int(nbytes), int(kind), stream.handle), "hipMemcpyAsync")


def copy2d_async(dst, dpitch: int, src, spitch: int, width: int, height: int, kind: int,
                 stream: Stream) -> None:
    """`height` rows of `width` bytes, row pitches `dpitch` / `spitch` (hipMemcpy2DAsync)."""
    check(hip().hipMemcpy2DAsync(dst, int(dpitch), src, int(spitch), int(width), int(height),
                                 int(kind), stream.handle), "hipMemcpy2DAsync")
