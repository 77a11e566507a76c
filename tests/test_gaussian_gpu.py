"""GPU parity of the Gaussian (gaussian.hip through the C ABI) against the oracle: bit-exact, as
the passes follow the reference's f32 operation order (gaussian.rs:110-119, kernel.rs:17-73)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.gpu_util import from_dev, to_dev
from tests.test_gaussian import KAT_IN, KAT_OUT

pytestmark = pytest.mark.gpu

import zarrs_tools_amd as zt  # noqa: E402  (no skip: the HIP library must load)
from zarrs_tools_amd import store as S  # noqa: E402


def gpu_gaussian(v, din, dout, chunk, sigma, half):
    import torch
    x = to_dev(v, din)
    y = torch.empty(v.shape, dtype=zt.torch_dtype(dout), device="cuda")
    zt.Gaussian(sigma, half).apply(zt.DeviceArray(x, chunk, din), zt.DeviceArray(y, chunk, dout))
    torch.cuda.synchronize()
    return from_dev(y, dout)


def test_reference_kat_bit_exact():
    out = gpu_gaussian(KAT_IN, "float32", "float32", (2, 2), [1.0, 1.0], [3, 3])
    assert np.array_equal(out, KAT_OUT)


@pytest.mark.parametrize("shape,chunk,sigma,half", [
    ((300,), (64,), [2.0], [6]),
    ((33, 70), (16, 32), [1.0, 1.5], [3, 5]),
    ((19, 37, 70), (8, 16, 32), [1.0, 1.0, 1.0], [3, 3, 3]),
    ((12, 20, 41), (5, 7, 9), [0.0, 2.2, 0.6], [2, 7, 2]),
    ((6, 7, 8, 9), (3, 4, 4, 5), [0.9, 1.1, 1.3, 0.7], [2, 3, 4, 2]),
])
def test_matches_oracle_bit_exactly(shape, chunk, sigma, half):
    rng = np.random.default_rng(sum(shape))
    v = (rng.random(shape, dtype=np.float32) * 1000 - 200).astype(np.float32)
    ref = O.gaussian_apply(v, chunk, sigma, half)
    out = gpu_gaussian(v, "float32", "float32", chunk, sigma, half)
    assert np.array_equal(out, ref)


def test_per_chunk_path_and_subset():
    import torch
    v = O.synth_step_noise_f32((14, 30, 50))
    sigma, half, chunk = [1.0, 2.0, 1.5], [3, 6, 4], (5, 16, 20)
    ref = O.gaussian_apply(v, chunk, sigma, half)
    x = to_dev(v, "float32")
    y = torch.empty(v.shape, device="cuda")
    a_in, a_out = zt.DeviceArray(x, chunk), zt.DeviceArray(y, chunk)
    g = zt.Gaussian(sigma, half)
    import itertools
    for idx in itertools.product(*[range(n) for n in a_out.chunk_grid_shape()]):
        g.apply_chunk(a_in, a_out, idx)
    torch.cuda.synchronize()
    assert np.array_equal(from_dev(y, "float32"), ref)


@pytest.mark.parametrize("din", list(O.DTYPES))
def test_all_input_types(din):
    rng = np.random.default_rng(3)
    v32 = (rng.random((6, 11, 40), dtype=np.float32) * 200 - (50 if din.startswith("int") else 0))
    v = O.cast_from_f32(v32, din)
    ref = O.gaussian_apply(O.cast_to_f32(v, din), (4, 8, 16), [1.0, 1.2, 0.8], [3, 4, 2])
    out = gpu_gaussian(v, din, "float32", (4, 8, 16), [1.0, 1.2, 0.8], [3, 4, 2])
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("dout", list(O.DTYPES))
def test_all_output_types(dout):
    v = O.synth_step_noise_f32((6, 11, 40)) * np.float32(0.4)
    ref = O.gaussian_apply(v, (4, 8, 16), [1.0, 1.0, 1.0], [3, 3, 3])
    out = gpu_gaussian(v, "float32", dout, (4, 8, 16), [1.0, 1.0, 1.0], [3, 3, 3])
    want = O.cast_from_f32(ref, dout)
    assert np.array_equal(out.view(np.uint8), want.view(np.uint8))


# Quad staging of the fused march (gauss_zyx_kernel<.., QUAD>): x extent a multiple of 4, several
# x tiles with edge quads on both sides, 1/2/4-byte inputs, the 128-VGPR form (L = 7) and the
# widest margin (L = 13).
@pytest.mark.parametrize("din", ["float32", "uint16", "uint8"])
@pytest.mark.parametrize("half", [3, 6])
def test_fused_zyx_quad_staging_bit_exact(din, half):
    rng = np.random.default_rng(7 + half)
    v32 = (rng.random((9, 37, 264), dtype=np.float32) * 250).astype(np.float32)
    v = O.cast_from_f32(v32, din)
    chunk = (9, 37, 264)
    ref = O.gaussian_apply(O.cast_to_f32(v, din), chunk, [1.0, 1.3, 0.9], [half] * 3)
    out = gpu_gaussian(v, din, "float32", chunk, [1.0, 1.3, 0.9], [half] * 3)
    assert np.array_equal(out, ref)


# Wide tiles of the fused march (ZYXWide, 32 x 256 on 1024 threads: quad marches with L <= 7 over
# blocks at least 256 wide): several x tiles with a partial last one, chunk regions starting at
# x = 300 (quad-aligned, not tile-aligned), partial y tiles, L = 3, 5 and 7, 1/2/4-byte inputs.
@pytest.mark.parametrize("din,half", [("float32", 1), ("float32", 2), ("float32", 3),
                                      ("uint16", 3), ("uint8", 2)])
def test_fused_zyx_wide_tiles_bit_exact(din, half):
    rng = np.random.default_rng(11 + half)
    shape, chunk = (21, 70, 600), (21, 35, 300)
    v32 = (rng.random(shape, dtype=np.float32) * 250).astype(np.float32)
    v = O.cast_from_f32(v32, din)
    sigma = [1.0, 1.3, 0.9]
    ref = O.gaussian_apply(O.cast_to_f32(v, din), chunk, sigma, [half] * 3)
    out = gpu_gaussian(v, din, "float32", chunk, sigma, [half] * 3)
    assert np.array_equal(out, ref)
    # chunk by chunk (regions at x = 0 and x = 300)
    import itertools
    import torch
    x = to_dev(v, din)
    y = torch.empty(shape, device="cuda")
    a_in, a_out = zt.DeviceArray(x, chunk, din), zt.DeviceArray(y, chunk)
    g = zt.Gaussian(sigma, [half] * 3)
    for idx in itertools.product(*[range(n) for n in a_out.chunk_grid_shape()]):
        g.apply_chunk(a_in, a_out, idx)
    torch.cuda.synchronize()
    assert np.array_equal(from_dev(y, "float32"), ref)


# The fused z/y/x march (gaussian.hip gauss_zyx_kernel): one tap length L on the last three
# axes, L in 3..13; several tiles, z segments and chunk-region offsets.
@pytest.mark.parametrize("shape,chunk,sigma,half", [
    ((19, 37, 70), (8, 16, 32), [0.6] * 3, [1] * 3),
    ((70, 45, 150), (32, 32, 64), [1.0, 1.2, 0.9], [2, 2, 2]),
    ((90, 66, 130), (64, 33, 65), [1.0] * 3, [3] * 3),
    ((40, 35, 100), (16, 16, 32), [2.0] * 3, [4] * 3),
    ((30, 40, 70), (30, 40, 70), [2.5] * 3, [5] * 3),
    ((25, 31, 67), (7, 9, 11), [3.0] * 3, [6] * 3),
    ((3, 9, 20, 70), (2, 5, 8, 32), [1.0, 1.0, 0.8, 1.1], [2, 3, 3, 3]),
])
def test_fused_zyx_march_bit_exact(shape, chunk, sigma, half):
    rng = np.random.default_rng(sum(shape) + half[-1])
    v = (rng.random(shape, dtype=np.float32) * 1000 - 200).astype(np.float32)
    ref = O.gaussian_apply(v, chunk, sigma, half)
    out = gpu_gaussian(v, "float32", "float32", chunk, sigma, half)
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("din", ["uint8", "int16", "uint16", "float64"])
def test_fused_zyx_march_input_types(din):
    rng = np.random.default_rng(5)
    v32 = (rng.random((20, 24, 72), dtype=np.float32) * 200 - (50 if din.startswith("int") else 0))
    v = O.cast_from_f32(v32, din)
    ref = O.gaussian_apply(O.cast_to_f32(v, din), (8, 16, 32), [1.0] * 3, [3] * 3)
    out = gpu_gaussian(v, din, "float32", (8, 16, 32), [1.0] * 3, [3] * 3)
    assert np.array_equal(out, ref)


def test_fused_zyx_march_per_chunk():
    import itertools
    import torch
    v = O.synth_step_noise_f32((40, 48, 100))
    sigma, half, chunk = [1.0] * 3, [3] * 3, (16, 16, 32)
    ref = O.gaussian_apply(v, chunk, sigma, half)
    x = to_dev(v, "float32")
    y = torch.empty(v.shape, device="cuda")
    a_in, a_out = zt.DeviceArray(x, chunk), zt.DeviceArray(y, chunk)
    g = zt.Gaussian(sigma, half)
    for idx in itertools.product(*[range(n) for n in a_out.chunk_grid_shape()]):
        g.apply_chunk(a_in, a_out, idx)
    torch.cuda.synchronize()
    assert np.array_equal(from_dev(y, "float32"), ref)


@pytest.mark.parametrize("codec", ["bytes", "gzip"])
def test_store_gaussian(tmp_path, codec):
    shape, chunk = (40, 36, 70), (16, 16, 32)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, chunk,
                   None if codec == "bytes" else S.codecs_json(codec))
    S.write_array(tmp_path / "in.zarr", u)
    st = S.gaussian(tmp_path / "in.zarr", tmp_path / "out.zarr", [1.0, 1.5, 2.0], [3, 5, 6],
                    data_type="float32")
    ref = O.gaussian_apply(u.astype(np.float32), chunk, [1.0, 1.5, 2.0], [3, 5, 6])
    assert np.array_equal(S.read_array(tmp_path / "out.zarr"), ref)
    assert st["voxels"] == u.size


def test_zarrs_ome_gaussian_levels(tmp_path):
    from zarrs_tools_amd import zarrs_ome as ZO
    shape, chunk = (40, 36, 70), (16, 16, 32)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, chunk)
    S.write_array(tmp_path / "in.zarr", u)
    ZO.run(str(tmp_path / "in.zarr"), str(tmp_path / "ome"), max_levels=3,
           gaussian_sigma=[1.0, 1.0, 1.0], log=lambda *a: None)
    want = u
    for lvl in (1, 2, 3):
        g = O.gaussian_apply_ndarray(want.astype(np.float32), [1.0] * 3, [3] * 3)
        want = O.downsample(g, "float32", (2, 2, 2), "uint16")
        np.testing.assert_array_equal(S.read_array(tmp_path / "ome" / str(lvl)), want)
    import json
    ms = json.load(open(tmp_path / "ome" / "zarr.json"))["attributes"]["ome"]["multiscales"][0]
    assert ms["type"] == "gaussian"
