"""ctypes binding of the C ABI (include/zarrs_tools_amd.h) exported by libzarrs_tools_amd.so.

The library is built in-tree (``zarrs_tools_amd/csrc/Makefile`` -> ``zarrs_tools_amd/
libzarrs_tools_amd.so``). There is no fallback: if the library is missing or fails to load,
importing this module raises, so a GPU run can never silently take a CPU path.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libzarrs_tools_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "zarrs_tools_amd.h")

# zt_status
OK = 0
ERR_INVALID_PARAMETERS = -1
ERR_UNSUPPORTED_DATA_TYPE = -2
ERR_OUT_OF_MEMORY = -3
ERR_DEVICE = -4
ERR_STORAGE = -5
ERR_ARRAY = -6
ERR_IO = -7
ERR_JSON = -8
ERR_INCOMPATIBLE_FILL_VALUE = -9
ERR_OTHER = -10

# zt_dtype (Zarr V3 data type names, guided_filter.rs:208-222)
DTYPES = {
    "bool": 0, "int8": 1, "int16": 2, "int32": 3, "int64": 4,
    "uint8": 5, "uint16": 6, "uint32": 7, "uint64": 8,
    "bfloat16": 9, "float16": 10, "float32": 11, "float64": 12,
}
DTYPE_NAMES = {v: k for k, v in DTYPES.items()}


class FilterError(RuntimeError):
    """Mirror of the reference's FilterError (src/filter/filter_error.rs:10-30)."""

    def __init__(self, status: int, message: str):
        super().__init__(f"{message} (status {status})")
        self.status = status


class InvalidParameters(FilterError):
    pass


class UnsupportedDataType(FilterError):
    pass


class DeviceError(FilterError):
    pass


_STATUS_CLASS = {
    ERR_INVALID_PARAMETERS: InvalidParameters,
    ERR_UNSUPPORTED_DATA_TYPE: UnsupportedDataType,
    ERR_DEVICE: DeviceError,
}

_lib = None

# flags of the store filters
STORE_ERASE_OUTPUT_METADATA = 1
STORE_FINISH_OUTPUT = 2


class Progress(ctypes.Structure):
    """zt_progress (include/zarrs_tools_amd.h): Progress stats of progress.rs:6-13."""
    _fields_ = [("step", ctypes.c_int64), ("num_steps", ctypes.c_int64),
                ("read_s", ctypes.c_double), ("process_s", ctypes.c_double),
                ("write_s", ctypes.c_double)]


PROGRESS_FN = ctypes.CFUNCTYPE(None, ctypes.POINTER(Progress), ctypes.c_void_p)


class StoreStats(ctypes.Structure):
    """zt_store_stats (include/zarrs_tools_amd.h)."""
    _fields_ = [("wall_s", ctypes.c_double), ("decode_s", ctypes.c_double),
                ("encode_s", ctypes.c_double), ("h2d_s", ctypes.c_double),
                ("kernel_s", ctypes.c_double), ("d2h_s", ctypes.c_double),
                ("bytes_read", ctypes.c_uint64), ("bytes_written", ctypes.c_uint64),
                ("voxels", ctypes.c_uint64), ("rows", ctypes.c_int64), ("threads", ctypes.c_int),
                ("rows_in_flight", ctypes.c_int), ("double_buffered", ctypes.c_int)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


def header_symbols() -> list[str]:
    """Every function name declared in include/zarrs_tools_amd.h."""
    text = open(HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(zt_[a-z0-9_]+)\s*\(", text)))


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C zarrs_tools_amd/csrc` "
            "(or __graft_entry__.build()). There is no CPU fallback.")
    # torch ships its own libamdhip64 (same soname). Load it first so the process has exactly
    # one HIP runtime: our NEEDED libamdhip64.so.7 then binds to the already-loaded copy. A
    # process that never uses torch (ZT_NO_TORCH=1: zarrs_ome's octant workers, hiprt.py) skips
    # it and binds the ROCm runtime of the library's RUNPATH.
    if os.environ.get("ZT_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(LIB_PATH)
    i64p = ctypes.POINTER(ctypes.c_int64)
    vp = ctypes.c_void_p
    c_int, c_float = ctypes.c_int, ctypes.c_float
    fp = ctypes.POINTER(ctypes.c_float)
    sig = {
        "zt_abi_version": ([], c_int),
        "zt_last_error": ([], ctypes.c_char_p),
        "zt_dtype_size": ([c_int], ctypes.c_size_t),
        "zt_device_count": ([ctypes.POINTER(c_int)], c_int),
        "zt_ctx_create": ([c_int, ctypes.POINTER(vp)], c_int),
        "zt_ctx_destroy": ([vp], c_int),
        "zt_ctx_set_stream": ([vp, vp], c_int),
        "zt_ctx_get_stream": ([vp, ctypes.POINTER(vp)], c_int),
        "zt_ctx_use_own_stream": ([vp], c_int),
        "zt_ctx_synchronize": ([vp], c_int),
        "zt_ctx_scratch_bytes": ([vp, ctypes.POINTER(ctypes.c_uint64)], c_int),
        "zt_ctx_release_scratch": ([vp], c_int),
        "zt_ctx_last_kernel_ms": ([vp, ctypes.POINTER(c_float)], c_int),
        "zt_guided_filter_is_compatible": ([c_int, c_int], c_int),
        "zt_guided_filter_memory_per_chunk": ([c_int, c_int, i64p, c_int,
                                               ctypes.POINTER(ctypes.c_uint64)], c_int),
        "zt_subset_overlap": ([i64p, c_int, i64p, i64p, i64p, i64p, i64p, i64p], c_int),
        "zt_guided_filter_apply_ndarray": ([vp, c_int, vp, i64p, i64p, c_int, i64p, i64p, c_int,
                                            vp, i64p, c_float, c_int], c_int),
        "zt_guided_filter_apply_array": ([vp, c_int, vp, c_int, vp, i64p, c_int, i64p, c_float,
                                          c_int, i64p, i64p], c_int),
        "zt_guided_filter_apply_slab": ([vp, c_int, vp, c_int, vp, i64p, ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, i64p,
                                         c_float, c_int], c_int),
        "zt_downsample_is_compatible": ([c_int, c_int, c_int], c_int),
        "zt_downsample_output_shape": ([i64p, c_int, i64p, i64p], c_int),
        "zt_downsample_input_subset": ([i64p, c_int, i64p, i64p, i64p, i64p, i64p], c_int),
        "zt_downsample_apply_ndarray": ([vp, c_int, vp, i64p, c_int, i64p, c_int, c_int, vp],
                                        c_int),
        "zt_pyramid_level_shapes": ([i64p, c_int, i64p, c_int, i64p, ctypes.POINTER(c_int)],
                                    c_int),
        "zt_pyramid_downsample": ([vp, c_int, vp, i64p, c_int, i64p, c_int, c_int,
                                   ctypes.POINTER(vp), ctypes.POINTER(c_int)], c_int),
        "zt_gaussian_kernel": ([c_float, ctypes.c_int64, fp, i64p], c_int),
        "zt_gaussian_is_compatible": ([c_int, c_int], c_int),
        "zt_gaussian_memory_per_chunk": ([c_int, c_int, i64p, c_int, i64p,
                                          ctypes.POINTER(ctypes.c_uint64)], c_int),
        "zt_gaussian_apply_ndarray": ([vp, c_int, vp, i64p, c_int, i64p, i64p, c_int, vp, fp,
                                       i64p], c_int),
        "zt_gaussian_apply_array": ([vp, c_int, vp, c_int, vp, i64p, c_int, i64p, fp, i64p],
                                    c_int),
        "zt_synth_step_noise_f32": ([vp, vp, i64p, c_int, i64p, ctypes.c_int64, ctypes.c_uint64],
                                    c_int),
        "zt_synth_u16": ([vp, vp, i64p, c_int, i64p, ctypes.c_int64, ctypes.c_uint64], c_int),
        "zt_reencode_cast": ([vp, c_int, vp, c_int, vp, ctypes.c_int64], c_int),
        "zt_synth_box": ([vp, c_int, vp, i64p, i64p, i64p, c_int, ctypes.c_uint64], c_int),
        # store -> store path (host storage)
        "zt_store_array_info": ([ctypes.c_char_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                 i64p, i64p, i64p], c_int),
        "zt_store_create_array": ([ctypes.c_char_p, c_int, c_int, i64p, i64p, ctypes.c_char_p,
                                   ctypes.c_char_p], c_int),
        "zt_store_create_output": ([ctypes.c_char_p, ctypes.c_char_p, c_int, i64p, c_int,
                                    ctypes.c_char_p], c_int),
        "zt_store_create_output_like": ([ctypes.c_char_p, ctypes.c_char_p, c_int,
                                         ctypes.c_char_p], c_int),
        "zt_store_set_progress_callback": ([PROGRESS_FN, vp], None),
        "zt_store_set_chunk_limit": ([ctypes.c_int64], ctypes.c_int),
        "zt_store_read_subset": ([ctypes.c_char_p, i64p, i64p, vp, c_int], c_int),
        "zt_store_write_subset": ([ctypes.c_char_p, i64p, i64p, vp, c_int], c_int),
        "zt_store_write_synth": ([ctypes.c_char_p, c_int, ctypes.c_uint64, c_int], c_int),
        "zt_store_guided_filter": ([ctypes.c_char_p, ctypes.c_char_p, c_int, ctypes.c_char_p,
                                    c_float, c_int, c_int, ctypes.c_int64, ctypes.c_int64, c_int,
                                    c_int, ctypes.POINTER(StoreStats)], c_int),
        "zt_store_guided_filter_box": ([ctypes.c_char_p, ctypes.c_char_p, c_int, ctypes.c_char_p,
                                        c_float, c_int, c_int, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_int64, c_int, c_int,
                                        ctypes.POINTER(StoreStats)], c_int),
        "zt_store_downsample": ([ctypes.c_char_p, ctypes.c_char_p, i64p, c_int, c_int,
                                 ctypes.c_char_p, c_int, ctypes.c_int64, ctypes.c_int64, c_int,
                                 c_int, ctypes.POINTER(StoreStats)], c_int),
        "zt_store_gaussian": ([ctypes.c_char_p, ctypes.c_char_p, c_int, ctypes.c_char_p, fp, i64p,
                               c_int, ctypes.c_int64, ctypes.c_int64, c_int, c_int,
                               ctypes.POINTER(StoreStats)], c_int),
        "zt_store_downsample_gaussian": ([ctypes.c_char_p, ctypes.c_char_p, i64p, fp, i64p, c_int,
                                          ctypes.c_char_p, c_int, ctypes.c_int64, ctypes.c_int64,
                                          c_int, c_int, ctypes.POINTER(StoreStats)], c_int),
        "zt_store_codec_available": ([ctypes.c_char_p], c_int),
        "zt_store_host_available_bytes": ([], ctypes.c_uint64),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(status: int) -> None:
    if status != OK:
        msg = lib().zt_last_error().decode(errors="replace")
        raise _STATUS_CLASS.get(status, FilterError)(status, msg)


def i64_array(values) -> ctypes.Array:
    vals = [int(v) for v in values]
    return (ctypes.c_int64 * max(len(vals), 1))(*vals)
