"""GPU parity: downsample (downsample.rs:72-120) and the device-resident zarrs_ome pyramid.
Same f64 sums in the same order as the reference restatement, so results are bit-exact."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.gpu_util import from_dev, to_dev

import zarrs_tools_amd as zt  # noqa: E402  (no skip: the HIP library must load)

pytestmark = pytest.mark.gpu


def gpu_ds(v, din, stride, dout, discrete=False):
    import torch
    x = to_dev(v, din)
    d = zt.Downsample(stride, discrete)
    y = d.apply_ndarray_discrete(x, dout) if discrete else d.apply_ndarray_continuous(x, dout)
    torch.cuda.synchronize()
    return from_dev(y, dout)


def test_golden(golden_cases, golden_dir):
    for c in golden_cases["downsample"]:
        vin = np.load(os.path.join(golden_dir, c["name"] + "_in.npy"))
        exp = np.load(os.path.join(golden_dir, c["name"] + "_out.npy"))
        out = gpu_ds(vin, c["dtype_in"], c["stride"], c["dtype_out"], c["discrete"])
        assert out.shape == exp.shape and np.array_equal(out, exp), c["name"]


@pytest.mark.parametrize("din", list(O.DTYPES))
@pytest.mark.parametrize("dout", list(O.DTYPES))
def test_all_type_pairs_bit_exact(din, dout):
    rng = np.random.default_rng(O.DTYPES[din] * 13 + O.DTYPES[dout])
    v32 = (rng.random((9, 10, 13)) * 250 - (100 if din.startswith("int") else 0)).astype(
        np.float32)
    v = O.cast_from_f32(v32, din)
    for stride in [(2, 2, 2), (3, 2, 4)]:
        ref = O.downsample(v, din, stride, dout)
        out = gpu_ds(v, din, stride, dout)
        assert np.array_equal(out, ref), (din, dout, stride)


@pytest.mark.parametrize("din", ["bool", "int8", "int16", "int32", "int64", "uint8", "uint16",
                                 "uint32", "uint64"])
def test_discrete_mode(din):
    rng = np.random.default_rng(3)
    v = O.cast_from_f32((rng.random((8, 9, 10)) * 4).astype(np.float32), din)
    ref = O.downsample(v, din, (2, 2, 2), din, discrete=True)
    out = gpu_ds(v, din, (2, 2, 2), din, discrete=True)
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("din,dout", [("int64", "int64"), ("uint64", "uint64"),
                                      ("int64", "float32"), ("uint64", "float64"),
                                      ("int64", "int32")])
def test_discrete_mode_64bit_beyond_2pow53(din, dout):
    """downsample.rs:113-117 counts exact TIn keys: 64-bit values past 2^53 that share one f64
    image stay distinct, the winner is returned exactly (or rounded once by `as` for float
    outputs, wrapped for narrower integers). Per-level kernel (2x2x2) and the N-d kernel (3x1x2)."""
    rng = np.random.default_rng(11)
    base = np.array([2 ** 62, 2 ** 62 + 1, 2 ** 62 + 3, 2 ** 62 + 2 ** 11, 2 ** 53 + 1],
                    dtype=np.uint64)
    if din == "int64":
        base = np.concatenate([base.astype(np.int64), -base.astype(np.int64)[:3]])
    v = base[rng.integers(0, len(base), (8, 10, 12))].astype(din)
    for stride in [(2, 2, 2), (3, 1, 2)]:
        ref = O.downsample(v, din, stride, dout, discrete=True)
        out = gpu_ds(v, din, stride, dout, discrete=True)
        np.testing.assert_array_equal(out, ref)


def test_discrete_rejects_float():
    import torch
    with pytest.raises(zt.UnsupportedDataType):
        zt.Downsample((2, 2), True).apply_ndarray_discrete(torch.zeros((4, 4), device="cuda"))


def test_whole_array_equals_per_chunk_reference_shape():
    # Downsample::apply reads input_subset(output chunk) per chunk; with complete windows only
    # the union equals the whole-array result. Check against the oracle chunk by chunk.
    import itertools
    import torch
    shape, stride, chunk = (37, 30, 41), (2, 2, 2), (7, 8, 9)
    v = O.synth_u16(shape)
    d = zt.Downsample(stride)
    oshape = d.output_shape(shape)
    x = to_dev(v, "uint16")
    y = torch.empty(oshape, dtype=torch.uint16, device="cuda")
    d.apply(zt.DeviceArray(x, chunk), zt.DeviceArray(y, chunk))
    torch.cuda.synchronize()
    out = from_dev(y, "uint16")
    grid = [-(-o // c) for o, c in zip(oshape, chunk)]
    for idx in itertools.product(*[range(g) for g in grid]):
        os_ = [i * c for i, c in zip(idx, chunk)]
        osh = [min(s + c, o) - s for s, c, o in zip(os_, chunk, oshape)]
        sub = d.input_subset(shape, zt.ArraySubset(tuple(os_), tuple(osh)))
        blk = v[tuple(slice(s, s + n) for s, n in zip(sub.start, sub.shape))]
        ref = O.downsample(blk, "uint16", stride, "uint16")
        got = out[tuple(slice(s, s + n) for s, n in zip(os_, osh))]
        assert np.array_equal(got, ref), idx


def test_pyramid_levels_bit_exact():
    import torch
    v = O.synth_u16((64, 48, 80))
    x = to_dev(v, "uint16")
    levels = zt.pyramid(x, (2, 2, 2), max_levels=5)
    torch.cuda.synchronize()
    assert [tuple(l.shape) for l in levels] == zt.pyramid_level_shapes(v.shape, (2, 2, 2), 5)
    cur = v
    for lvl in levels:
        cur = O.downsample(cur, "uint16", (2, 2, 2), "uint16")
        assert np.array_equal(from_dev(lvl, "uint16"), cur)


@pytest.mark.parametrize("shape,dtype", [
    ((37, 50, 71), "uint16"), ((64, 64, 64), "uint8"), ((9, 17, 33), "int16"),
    ((40, 36, 72), "float32"), ((24, 20, 16), "float64"), ((19, 32, 40), "int64"),
    ((16, 16, 264), "uint32"), ((70, 8, 8), "int8"), ((5, 300, 9), "uint16"),
    # u8 / bool take pyramid3_u8_mean_kernel (16-byte rows, dot4 sums): aligned rows with partial
    # lanes, rows that are not whole 16-byte quads, odd extents
    ((33, 34, 35), "uint8"), ((12, 8, 160), "uint8"), ((18, 20, 40), "uint8"),
    ((16, 12, 1056), "uint8"), ((33, 34, 35), "bool"), ((12, 8, 160), "int8"),
    ((33, 34, 35), "int8")])
def test_fused_pyramid_levels_equal_per_level_launches(shape, dtype, monkeypatch):
    """zt_pyramid_downsample fuses up to three 2x2x2 mean levels per launch; every level must be
    bit-identical to the oracle's level-by-level downsample (odd extents, partial workgroups,
    unaligned rows, 8- to 64-bit types) and to the unfused launches."""
    import torch
    rng = np.random.default_rng(sum(shape))
    if dtype == "bool":
        v = rng.integers(0, 2, shape).astype(bool)
    elif dtype.startswith("float"):
        v = (rng.standard_normal(shape) * 1000.0).astype(dtype)
    else:
        info = np.iinfo(dtype)
        v = rng.integers(info.min, info.max, shape, dtype=dtype, endpoint=True)
    x = to_dev(v, dtype)
    levels = zt.pyramid(x, (2, 2, 2), max_levels=6)
    # the per-level launches: one Downsample::apply_ndarray_continuous per level
    plain, cur_dev = [], x
    for _ in levels:
        cur_dev = zt.Downsample((2, 2, 2)).apply_ndarray_continuous(cur_dev)
        plain.append(cur_dev)
    torch.cuda.synchronize()
    assert len(levels) == len(zt.pyramid_level_shapes(shape, (2, 2, 2), 6))
    cur = v
    for got, ref in zip(levels, plain):
        cur = O.downsample(cur, dtype, (2, 2, 2), dtype)
        g = from_dev(got, dtype)
        assert g.shape == cur.shape
        np.testing.assert_array_equal(g, cur)
        np.testing.assert_array_equal(g, from_dev(ref, dtype))


@pytest.mark.parametrize("shape,dtype,levels", [
    ((37, 50, 71), "uint16", 6), ((64, 64, 64), "uint8", 6), ((9, 17, 33), "int16", 6),
    ((19, 32, 40), "int64", 6), ((16, 16, 264), "uint32", 6), ((70, 8, 8), "int8", 6),
    ((33, 34, 35), "bool", 6), ((40, 36, 72), "int32", 2),
    # the packed-byte kernel (pyramid3_u8_kernel): 16-byte rows with partial lanes, odd extents
    ((12, 8, 160), "uint8", 4), ((33, 34, 35), "uint8", 6), ((12, 8, 160), "int8", 4),
    ((33, 34, 35), "int8", 6), ((16, 16, 96), "bool", 4)])
def test_fused_mode_pyramid_equals_oracle_levels(shape, dtype, levels):
    """zarrs_ome --discrete on the device: the level-fused mode pyramid (pyr_mode8, up to three
    levels per launch) gives, level by level, the oracle's discrete downsample of the previous
    level (the most frequent value, ties to the smallest: the documented tie rule) and the
    per-level mode launches. Few distinct values so that ties and majorities both occur."""
    import torch
    rng = np.random.default_rng(sum(shape) + levels)
    if dtype == "bool":
        v = rng.integers(0, 2, shape).astype(bool)
    else:
        info = np.iinfo(dtype)
        # the full range: the oracle counts exact integer keys (64-bit values past 2^53 included)
        pool = rng.integers(info.min, info.max, 5, dtype=dtype, endpoint=True)
        v = pool[rng.integers(0, 5, shape)]
    x = to_dev(v, dtype)
    got_levels = zt.pyramid(x, (2, 2, 2), max_levels=levels, discrete=True)
    plain, cur_dev = [], x
    for _ in got_levels:
        cur_dev = zt.Downsample((2, 2, 2), discrete=True).apply_ndarray_discrete(cur_dev)
        plain.append(cur_dev)
    torch.cuda.synchronize()
    assert len(got_levels) == len(zt.pyramid_level_shapes(shape, (2, 2, 2), levels))
    cur = v
    for got, ref in zip(got_levels, plain):
        cur = O.downsample(cur, dtype, (2, 2, 2), dtype, discrete=True)
        g = from_dev(got, dtype)
        assert g.shape == cur.shape
        np.testing.assert_array_equal(g, cur)
        np.testing.assert_array_equal(g, from_dev(ref, dtype))


def test_pyramid_tall_y_beyond_the_fused_grid():
    """A level-1 y extent past 4 x 65535 rows does not fit the fused launch's grid: those levels
    take the per-level launches and still equal the oracle's level-by-level result."""
    import torch
    shape = (4, 4 * 65536 * 2 + 16, 4)  # level 1 y extent 262152 -> 65538 y workgroups
    rng = np.random.default_rng(7)
    v = rng.integers(0, 255, shape, dtype=np.uint8, endpoint=True)
    levels = zt.pyramid(to_dev(v, "uint8"), (2, 2, 2), max_levels=3)
    torch.cuda.synchronize()
    cur = v
    for lvl in levels:
        cur = O.downsample(cur, "uint8", (2, 2, 2), "uint8")
        np.testing.assert_array_equal(from_dev(lvl, "uint8"), cur)
