"""CPU: the C-ABI library loads, exports every symbol include/zarrs_tools_amd.h declares, and its
host-only entry points (no device work) behave like the reference's operator surface."""
import ctypes

import pytest

import zarrs_tools_amd as zt
from zarrs_tools_amd import _abi


def test_library_exports_every_header_symbol():
    names = _abi.header_symbols()
    assert len(names) >= 20
    lib = _abi.lib()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version():
    assert _abi.lib().zt_abi_version() == 4


def test_device_count_never_errors():
    n = ctypes.c_int(-1)
    assert _abi.lib().zt_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0


def test_dtype_sizes():
    sizes = {"bool": 1, "int8": 1, "int16": 2, "int32": 4, "int64": 8, "uint8": 1, "uint16": 2,
             "uint32": 4, "uint64": 8, "bfloat16": 2, "float16": 2, "float32": 4, "float64": 8}
    for name, sz in sizes.items():
        assert _abi.lib().zt_dtype_size(_abi.DTYPES[name]) == sz
    assert _abi.lib().zt_dtype_size(99) == 0


def test_is_compatible_all_13_types():
    g = zt.GuidedFilter(2500.0, 4)
    for a in _abi.DTYPES:
        for b in _abi.DTYPES:
            g.is_compatible(a, b)
    with pytest.raises(zt.UnsupportedDataType):
        g.is_compatible("complex64", "float32")
    with pytest.raises(zt.UnsupportedDataType):
        _abi.check(_abi.lib().zt_guided_filter_is_compatible(99, 11))


def test_downsample_discrete_rejects_floats():
    d = zt.Downsample([2, 2], discrete=True)
    d.is_compatible("uint8", "uint8")
    with pytest.raises(zt.UnsupportedDataType):
        d.is_compatible("float32", "float32")


def test_memory_per_chunk_matches_reference_formula():
    # guided_filter.rs:234-237
    g = zt.GuidedFilter(1.0, 2)
    assert g.memory_per_chunk("uint16", "float32", (256, 256, 256)) == 2 + 4 + 256 ** 3 * 16


def test_subset_overlap_clamps_at_array_edges():
    # array_subset_overlap.rs:11-35 with the guided filter's 2r halo
    o = zt.ArraySubsetOverlap((10, 20), zt.ArraySubset((0, 8), (4, 4)), (3, 3))
    assert o.subset_input() == zt.ArraySubset((0, 5), (7, 10))
    assert o.subset_dst_in_src() == zt.ArraySubset((0, 3), (4, 4))
    o = zt.ArraySubsetOverlap((10, 20), zt.ArraySubset((8, 16), (2, 4)), (3, 3))
    assert o.subset_input() == zt.ArraySubset((5, 13), (5, 7))


def test_subset_overlap_rejects_out_of_bounds():
    with pytest.raises(zt.InvalidParameters):
        zt.ArraySubsetOverlap((4,), zt.ArraySubset((3,), (2,)), (1,))


def test_downsample_shapes():
    d = zt.Downsample([2, 2, 2])
    assert d.output_shape((5, 1, 8)) == (2, 1, 4)
    s = d.input_subset((5, 1, 8), zt.ArraySubset((1, 0, 2), (1, 1, 2)))
    assert s == zt.ArraySubset((2, 0, 4), (2, 1, 4))
    with pytest.raises(zt.InvalidParameters):
        zt.Downsample([0, 2, 2]).output_shape((4, 4, 4))


def test_pyramid_shapes_and_stop_rule():
    # zarrs_ome.rs:515 + :731-737
    assert zt.pyramid_level_shapes((4096,) * 3, (2, 2, 2), 5) == [
        (2048,) * 3, (1024,) * 3, (512,) * 3, (256,) * 3, (128,) * 3]
    shapes = zt.pyramid_level_shapes((5, 8, 3), (2, 2, 2), 10)
    assert shapes == [(2, 4, 1), (1, 2, 1), (1, 1, 1)]
    # factor 1 on an axis: stop when the other axes reach 1
    assert zt.pyramid_level_shapes((4, 1), (2, 1), 10) == [(2, 1), (1, 1)]


def test_context_creation_fails_cleanly_without_gpu():
    n = ctypes.c_int()
    _abi.lib().zt_device_count(ctypes.byref(n))
    if n.value > 0:
        pytest.skip("GPU present")
    with pytest.raises(zt.FilterError):
        zt.Context(0)
    assert "device" in _abi.lib().zt_last_error().decode()


def test_radius_validation():
    n = ctypes.c_int()
    _abi.lib().zt_device_count(ctypes.byref(n))
    with pytest.raises(zt.InvalidParameters):
        zt.GuidedFilter(1.0, 300)
