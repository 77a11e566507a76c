"""zarrs_tools_amd — MI355X-native zarrs_filter per-chunk transform path.

The compute lives in libzarrs_tools_amd.so (hand-written HIP kernels for gfx950 behind the C ABI
in include/zarrs_tools_amd.h). This package is the thin host-side mirror of the reference's
filter-operator surface (LDeakin/zarrs_tools src/filter/) used by tests and bench.py.
Importing it loads the library; if it is missing the import fails loudly (no CPU fallback).
"""
from ._abi import DTYPES, FilterError, InvalidParameters, UnsupportedDataType, lib

lib()  # fail at import time if the native library is absent

from .filter import (  # noqa: E402
    ArraySubset,
    ArraySubsetOverlap,
    Context,
    DeviceArray,
    Downsample,
    Gaussian,
    GuidedFilter,
    default_context,
    dtype_of,
    pyramid,
    pyramid_level_shapes,
    synth_step_noise_f32,
    synth_u16,
    synth_box,
    torch_dtype,
)
from .shard import OctantAssignment, SlabAssignment, octant_assignment, slab_assignment  # noqa: E402

__all__ = [
    "ArraySubset", "ArraySubsetOverlap", "Context", "DeviceArray", "Downsample", "DTYPES",
    "FilterError", "Gaussian", "GuidedFilter", "InvalidParameters", "SlabAssignment", "UnsupportedDataType",
    "default_context", "dtype_of", "lib", "octant_assignment", "OctantAssignment", "pyramid",
    "pyramid_level_shapes", "slab_assignment",
    "synth_step_noise_f32", "synth_u16", "synth_box", "torch_dtype",
]
