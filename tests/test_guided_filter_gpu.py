"""GPU parity: the HIP guided filter (through the C ABI) against the oracle.

Tolerance: float outputs |gpu - oracle| <= 1e-5 * max(1, |oracle|); integer
outputs equal except where the f32 result sits within that tolerance of a truncation boundary.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.gpu_util import FLOAT_TOL, from_dev, rel_err, to_dev

pytestmark = pytest.mark.gpu

import zarrs_tools_amd as zt  # noqa: E402  (no skip: the HIP library must load)


def gpu_apply(v: np.ndarray, din: str, dout: str, chunk, eps, r):
    import torch
    x = to_dev(v, din)
    y = torch.empty(v.shape, dtype=zt.torch_dtype(dout), device="cuda")
    zt.GuidedFilter(eps, r).apply(zt.DeviceArray(x, chunk, din), zt.DeviceArray(y, chunk, dout))
    torch.cuda.synchronize()
    return from_dev(y, dout)


def gpu_apply_chunked(v: np.ndarray, din: str, dout: str, chunk, eps, r):
    """Reference-shaped path: every chunk reads its halo'd block and runs apply_ndarray."""
    import itertools
    import torch
    x = to_dev(v, din)
    y = torch.empty(v.shape, dtype=zt.torch_dtype(dout), device="cuda")
    a_in, a_out = zt.DeviceArray(x, chunk, din), zt.DeviceArray(y, chunk, dout)
    g = zt.GuidedFilter(eps, r)
    for idx in itertools.product(*[range(n) for n in a_out.chunk_grid_shape()]):
        g.apply_chunk(a_in, a_out, idx)
    torch.cuda.synchronize()
    return from_dev(y, dout)


def check_against(out, ref_f32, dout):
    if dout in ("float32", "float64"):
        assert rel_err(out, ref_f32) <= FLOAT_TOL
    elif dout in ("float16", "bfloat16"):
        ref = O.cast_from_f32(ref_f32, dout)
        o32 = O.cast_to_f32(out, dout).astype(np.float64)
        r32 = O.cast_to_f32(ref, dout).astype(np.float64)
        ulp = 2.0 ** -10 if dout == "float16" else 2.0 ** -7
        assert np.all(np.abs(o32 - r32) <= ulp * np.maximum(1.0, np.abs(r32)) + 1e-12)
    else:
        ref = O.cast_from_f32(ref_f32, dout)
        diff = out.astype(np.float64) != ref.astype(np.float64)
        if diff.any():
            # only where the f32 value is within tolerance of an integer boundary
            near = np.abs(ref_f32 - np.round(ref_f32)) <= FLOAT_TOL * np.maximum(1, np.abs(ref_f32))
            assert np.all(near[diff]), (np.argwhere(diff)[:5], ref_f32[diff][:5])
            assert np.all(np.abs(out.astype(np.float64) - ref.astype(np.float64))[diff] <= 1)


def test_reference_kat_through_c_abi():
    # guided_filter.rs:330-374: 4x4 f32, 2x2 chunks, eps 1, r 2
    v = np.array([[i + j for j in range(4)] for i in range(4)], dtype=np.float32)
    kat = np.array([[1.659829, 2.1910257, 2.5641026, 3.0],
                    [2.1910257, 2.614423, 3.0, 3.4358974],
                    [2.5641026, 3.0, 3.385577, 3.8089743],
                    [3.0, 3.4358974, 3.8089743, 4.340171]], dtype=np.float32)
    out = gpu_apply(v, "float32", "float32", (2, 2), 1.0, 2)
    assert rel_err(out, kat) <= FLOAT_TOL
    out2 = gpu_apply_chunked(v, "float32", "float32", (2, 2), 1.0, 2)
    assert rel_err(out2, kat) <= FLOAT_TOL
    print("KAT max abs diff", np.abs(out - kat).max(), "bit-exact", np.array_equal(out, kat))


def _golden(golden_dir, name, kind):
    return np.load(os.path.join(golden_dir, f"{name}_{kind}.npy"))


def test_golden_whole_array(golden_cases, golden_dir):
    for c in golden_cases["guided_filter"]:
        vin = _golden(golden_dir, c["name"], "in")
        ref = _golden(golden_dir, c["name"], "out_f32")
        out = gpu_apply(vin, c["dtype_in"], c["dtype_out"], c["chunk_shape"], c["epsilon"],
                        c["radius"])
        check_against(out, ref, c["dtype_out"])


def test_golden_per_chunk(golden_cases, golden_dir):
    for c in golden_cases["guided_filter"]:
        vin = _golden(golden_dir, c["name"], "in")
        ref = _golden(golden_dir, c["name"], "out_f32")
        out = gpu_apply_chunked(vin, c["dtype_in"], c["dtype_out"], c["chunk_shape"],
                                c["epsilon"], c["radius"])
        check_against(out, ref, c["dtype_out"])


@pytest.mark.parametrize("r", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 12])
def test_radii_3d(r):
    rng = np.random.default_rng(r)
    shape = (int(rng.integers(9, 30)), int(rng.integers(9, 70)), int(rng.integers(9, 90)))
    chunk = tuple(int(rng.integers(4, 20)) for _ in range(3))
    v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
    eps = float(rng.choice([0.5, 50.0, 2500.0]))
    ref = O.guided_filter_apply(v, chunk, eps, r, nthreads=8)
    out = gpu_apply(v, "float32", "float32", chunk, eps, r)
    assert rel_err(out, ref) <= FLOAT_TOL, (shape, chunk, eps)


def test_radius_zero_is_identity():
    v = O.synth_step_noise_f32((7, 9, 70))
    out = gpu_apply(v, "float32", "float32", (4, 4, 32), 2500.0, 0)
    assert np.array_equal(out, v)


@pytest.mark.parametrize("din", list(O.DTYPES))
def test_all_input_types(din):
    rng = np.random.default_rng(7)
    v32 = (rng.random((6, 13, 70), dtype=np.float32) * 200 - (50 if din.startswith("int") else 0))
    v = O.cast_from_f32(v32, din)
    ref = O.guided_filter_apply(O.cast_to_f32(v, din), (4, 8, 32), 100.0, 2, nthreads=8)
    out = gpu_apply(v, din, "float32", (4, 8, 32), 100.0, 2)
    assert rel_err(out, ref) <= FLOAT_TOL


# 8- and 16-bit integer inputs take the fused kernel's integer stage 1 (exact int32 window sums,
# 4-byte Hx rows): full-range values (W^3 * 65535 near 2^31 at r = 8), eps down to 0.5 (where a
# 1-ulp error in u shows), quad-aligned geometry (one mode-1 grid) and odd widths (masked edge
# tiles), whole array and chunk by chunk.
@pytest.mark.parametrize("din", ["uint16", "uint8"])
@pytest.mark.parametrize("r", [1, 2, 3, 4, 5, 8])
def test_integer_inputs_stage1_exact(din, r):
    rng = np.random.default_rng(100 + r)
    top = 65535 if din == "uint16" else 255
    for shape, chunk in [((12, 40, 136), (6, 16, 64)), ((11, 37, 91), (5, 13, 30))]:
        v = rng.integers(0, top + 1, size=shape).astype(din)
        for eps in (0.5, 2500.0):
            ref = O.guided_filter_apply(O.cast_to_f32(v, din), chunk, eps, r, nthreads=8)
            out = gpu_apply(v, din, "float32", chunk, eps, r)
            assert rel_err(out, ref) <= FLOAT_TOL, (shape, eps)
        out = gpu_apply_chunked(v, din, "float32", chunk, eps, r)
        assert rel_err(out, ref) <= FLOAT_TOL, (shape, "per chunk")


@pytest.mark.parametrize("dout", list(O.DTYPES))
def test_all_output_types(dout):
    v = O.synth_step_noise_f32((6, 13, 70)) * np.float32(0.4)
    ref = O.guided_filter_apply(v, (4, 8, 32), 100.0, 2, nthreads=8)
    out = gpu_apply(v, "float32", dout, (4, 8, 32), 100.0, 2)
    check_against(out, ref, dout)


def test_degenerate_shapes():
    for shape in [(0, 5, 5), (1, 1, 1), (1, 1, 300), (3, 1, 1), (1, 65, 1)]:
        v = O.synth_step_noise_f32(shape) if 0 not in shape else np.zeros(shape, np.float32)
        ref = O.guided_filter_apply(v, (2, 2, 64), 2500.0, 2) if v.size else v
        out = gpu_apply(v, "float32", "float32", (2, 2, 64), 2500.0, 2)
        assert out.shape == v.shape
        if v.size:
            assert rel_err(out, ref) <= FLOAT_TOL, shape


def test_subset_of_chunk_grid_only_touches_those_chunks():
    import torch
    v = O.synth_step_noise_f32((16, 16, 64))
    ref = O.guided_filter_apply(v, (8, 8, 32), 2500.0, 2)
    x = to_dev(v, "float32")
    y = torch.full(v.shape, -1.0, device="cuda")
    zt.GuidedFilter(2500.0, 2).apply(zt.DeviceArray(x, (8, 8, 32)), zt.DeviceArray(y, (8, 8, 32)),
                                     chunk_grid_start=(1, 0, 1), chunk_grid_count=(1, 2, 1))
    out = from_dev(y, "float32")
    assert rel_err(out[8:, :, 32:], ref[8:, :, 32:]) <= FLOAT_TOL
    assert np.all(out[:8] == -1) and np.all(out[:, :, :32] == -1)


def test_slab_form_equals_whole_array():
    import torch
    shape, chunk, r = (48, 40, 96), (16, 16, 32), 4
    v = O.synth_step_noise_f32(shape)
    whole = gpu_apply(v, "float32", "float32", chunk, 2500.0, r)
    x = to_dev(v, "float32")
    res = np.empty_like(v)
    for rank in range(3):
        a = zt.slab_assignment(rank, 3, shape[0], chunk[0], 2 * r)
        y = torch.empty((a.out_nz,) + shape[1:], device="cuda")
        slab = x[a.in_z0:a.in_z0 + a.in_nz].contiguous()
        zt._abi.check(zt._abi.lib().zt_guided_filter_apply_slab(
            zt.default_context().handle, 11, zt.filter._ptr(slab), 11, zt.filter._ptr(y),
            zt._abi.i64_array(shape), a.in_z0, a.in_nz, a.out_z0, a.out_nz,
            zt._abi.i64_array(chunk), 2500.0, r))
        torch.cuda.synchronize()
        res[a.out_z0:a.out_z0 + a.out_nz] = from_dev(y, "float32")
    assert np.array_equal(res, whole)


def test_synthetic_generator_matches_oracle():
    import torch
    shape = (5, 33, 70)
    d = zt.synth_step_noise_f32(shape, global_shape=(9, 33, 70), z0=3)
    torch.cuda.synchronize()
    assert np.array_equal(from_dev(d, "float32"),
                          O.synth_step_noise_f32(shape, global_shape=(9, 33, 70), z0=3))
    u = zt.synth_u16((4, 5, 6), z0=2, global_shape=(8, 5, 6))
    torch.cuda.synchronize()
    assert np.array_equal(from_dev(u, "uint16"), O.synth_u16((4, 5, 6), z0=2,
                                                             global_shape=(8, 5, 6)))


def test_256_cube_r4_vs_oracle():
    shape, chunk = (256, 256, 256), (128, 128, 128)
    v = O.synth_step_noise_f32(shape)
    ref = O.guided_filter_apply(v, chunk, 2500.0, 4, nthreads=16)
    out = gpu_apply(v, "float32", "float32", chunk, 2500.0, 4)
    err = rel_err(out, ref)
    exact = float(np.mean(out == ref))
    print(f"256^3 r=4: max rel err {err:.3e}, bit-exact fraction {exact:.4f}")
    assert err <= FLOAT_TOL


# ---- separable N-d path: 4-D / 5-D arrays and radii > 8 ---------------------

@pytest.mark.parametrize("r", [1, 2, 3, 8, 9, 12])
def test_separable_4d_vs_oracle_small_eps(r):
    """Exact f64 stage-1 sums: u matches the reference's even at eps = 0.5, where a 1-ulp error
    in u moves the output by ~1e-4 relative."""
    rng = np.random.default_rng(100 + r)
    shape = (int(rng.integers(3, 7)), int(rng.integers(5, 14)), int(rng.integers(5, 20)),
             int(rng.integers(5, 40)))
    chunk = tuple(int(rng.integers(2, 9)) for _ in range(4))
    v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
    ref = O.guided_filter_apply(v, chunk, 0.5, r, nthreads=8)
    out = gpu_apply(v, "float32", "float32", chunk, 0.5, r)
    assert rel_err(out, ref) <= FLOAT_TOL, (shape, chunk)


def test_separable_4d_whole_box_equals_per_chunk():
    v = O.synth_step_noise_f32((4, 12, 20, 36))
    chunk = (2, 8, 8, 16)
    whole = gpu_apply(v, "float32", "float32", chunk, 2500.0, 2)
    per_chunk = gpu_apply_chunked(v, "float32", "float32", chunk, 2500.0, 2)
    ref = O.guided_filter_apply(v, chunk, 2500.0, 2, nthreads=8)
    assert rel_err(whole, ref) <= FLOAT_TOL
    assert rel_err(per_chunk, ref) <= FLOAT_TOL


def test_separable_5d_and_u16_input():
    rng = np.random.default_rng(5)
    v32 = (rng.random((3, 4, 5, 6, 18), dtype=np.float32) * 200).astype(np.float32)
    v = O.cast_from_f32(v32, "uint16")
    chunk = (2, 2, 4, 4, 8)
    ref = O.guided_filter_apply(O.cast_to_f32(v, "uint16"), chunk, 50.0, 1, nthreads=8)
    out = gpu_apply(v, "uint16", "float32", chunk, 50.0, 1)
    assert rel_err(out, ref) <= FLOAT_TOL


@pytest.mark.parametrize("r", [2, 9])
def test_separable_4d_chunk_grid_subset(r):
    """A sub-box of the chunk grid: the whole-box launch reads only the box plus its halo and
    writes only the box."""
    import torch
    v = O.synth_step_noise_f32((4, 16, 16, 48))
    chunk = (2, 8, 8, 16)
    ref = O.guided_filter_apply(v, chunk, 2500.0, r, nthreads=8)
    x = to_dev(v, "float32")
    y = torch.full(v.shape, -1.0, device="cuda")
    zt.GuidedFilter(2500.0, r).apply(zt.DeviceArray(x, chunk), zt.DeviceArray(y, chunk),
                                     chunk_grid_start=(1, 0, 1, 1),
                                     chunk_grid_count=(1, 2, 1, 2))
    out = from_dev(y, "float32")
    box = (slice(2, 4), slice(0, 16), slice(8, 16), slice(16, 48))
    assert rel_err(out[box], ref[box]) <= FLOAT_TOL
    mask = np.ones(v.shape, bool)
    mask[box] = False
    assert np.all(out[mask] == -1)


# ---- 4-D path (guided4d.hip: t-window sums of per-timepoint 3-D box sums), config T ----------

@pytest.mark.parametrize("din,dout", [("uint16", "float32"), ("float32", "uint8"),
                                      ("int16", "float64"), ("float32", "bfloat16")])
def test_guided4d_element_types(din, dout):
    rng = np.random.default_rng(41)
    v32 = (rng.random((5, 9, 14, 70), dtype=np.float32) * 200).astype(np.float32)
    v = O.cast_from_f32(v32, din)
    chunk = (2, 4, 8, 32)
    ref = O.guided_filter_apply(O.cast_to_f32(v, din), chunk, 300.0, 2, nthreads=8)
    out = gpu_apply(v, din, dout, chunk, 300.0, 2)
    check_against(out, ref, dout)


@pytest.mark.parametrize("r", [1, 2, 4, 6])
def test_guided4d_per_chunk_and_small_eps(r):
    rng = np.random.default_rng(7 + r)
    shape = (int(rng.integers(2, 9)), int(rng.integers(5, 20)), int(rng.integers(5, 30)),
             int(rng.integers(5, 90)))
    chunk = tuple(int(rng.integers(2, 9)) for _ in range(4))
    v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
    ref = O.guided_filter_apply(v, chunk, 0.5, r, nthreads=8)
    assert rel_err(gpu_apply(v, "float32", "float32", chunk, 0.5, r), ref) <= FLOAT_TOL
    assert rel_err(gpu_apply_chunked(v, "float32", "float32", chunk, 0.5, r), ref) <= FLOAT_TOL


@pytest.mark.parametrize("shape,chunk,r", [
    ((20, 9, 14, 40), (4, 4, 8, 16), 2),     # a (t, z) block of config T: 16 + 2r timepoints
    ((32, 6, 7, 20), (8, 3, 7, 10), 3),      # TMAX = 32
    ((17, 10, 12, 33), (5, 5, 6, 11), 6),
    ((12, 8, 9, 30), (4, 4, 9, 15), 1),      # TMAX = 16
])
def test_guided4d_long_series_small_eps(shape, chunk, r):
    """The 4-D path for blocks of 5-32 timepoints: stage 1 as the t-march (r <= 2) or K1 +
    g4_tab (r 3-6) writing the t-window sums of (a, b), then box3_final (their box3 with the final
    stage in the march): whole box and per chunk equal
    the oracle at eps = 0.5 (exact stage 1)."""
    rng = np.random.default_rng(sum(shape) + r)
    v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
    ref = O.guided_filter_apply(v, chunk, 0.5, r, nthreads=8)
    assert rel_err(gpu_apply(v, "float32", "float32", chunk, 0.5, r), ref) <= FLOAT_TOL
    assert rel_err(gpu_apply_chunked(v, "float32", "float32", chunk, 0.5, r), ref) <= FLOAT_TOL


@pytest.mark.parametrize("r", [1, 2, 3])
def test_guided4d_z_ring_many_steps(r):
    """The box3 marches' z-window register ring (box3_ring: the leaving slice from registers,
    the march unrolled by 2r + 1) over a z extent of several ring turns that is no multiple of
    2r + 1, with a z segment start inside the array (output box), against the oracle."""
    rng = np.random.default_rng(100 + r)
    shape, chunk = (6, 37, 20, 70), (3, 8, 10, 35)
    v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
    ref = O.guided_filter_apply(v, chunk, 0.5, r, nthreads=8)
    assert rel_err(gpu_apply(v, "float32", "float32", chunk, 0.5, r), ref) <= FLOAT_TOL
    assert rel_err(gpu_apply_chunked(v, "float32", "float32", chunk, 0.5, r), ref) <= FLOAT_TOL


def test_guided4d_block_output_box_vs_oracle():
    """apply_ndarray on a halo'd (t, z) block with an interior output box (the config T share
    form, tools/bench_ops.py): equals the oracle's per-chunk result of the whole array."""
    from zarrs_tools_amd import shard
    import torch
    shape, chunk, r = (16, 20, 12, 40), (4, 5, 12, 40), 2
    rng = np.random.default_rng(3)
    v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
    ref = O.guided_filter_apply(v, chunk, 0.5, r, nthreads=8)
    for rank in range(4):
        a = shard.block_assignment(rank, 4, shape, chunk, 2 * r, (2, 2))
        blk = np.ascontiguousarray(v[tuple(slice(s, s + n) for s, n in zip(a.in_start, a.in_shape))])
        x = torch.from_numpy(blk).cuda()
        sub = zt.ArraySubset(tuple(o - i for o, i in zip(a.out_start, a.in_start)), a.out_shape)
        got = zt.GuidedFilter(0.5, r).apply_ndarray(x, sub).cpu().numpy()
        want = ref[tuple(slice(o, o + n) for o, n in zip(a.out_start, a.out_shape))]
        assert rel_err(got, want) <= FLOAT_TOL, rank


@pytest.mark.parametrize("r", [1, 2])
def test_guided4d_tmarch_output_box_after_nan_scratch(r):
    """The t-march (g4_tmarch_tab_kernel, r <= 2, T > 4) writes TAB only on the output box + r,
    while box3_final reads whole tiles: the context scratch is first filled with NaN (a NaN
    input's U3 / TAB), then an interior output box of a clean block must still equal the oracle
    (stale scratch must never reach a stored output)."""
    import torch
    shape, chunk = (10, 24, 20, 72), (5, 8, 10, 24)
    poison = torch.full(shape, float("nan"), dtype=torch.float32, device="cuda")
    zt.GuidedFilter(0.5, r).apply_ndarray(poison)  # the default context: its scratch persists
    torch.cuda.synchronize()
    rng = np.random.default_rng(40 + r)
    v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
    ref = O.guided_filter_apply(v, chunk, 0.5, r, nthreads=8)
    sub = zt.ArraySubset((3, 5, 4, 9), (4, 11, 9, 50))  # interior in every axis
    got = zt.GuidedFilter(0.5, r).apply_ndarray(torch.from_numpy(v).cuda(), sub)
    torch.cuda.synchronize()
    want = ref[tuple(slice(s, s + n) for s, n in zip(sub.start, sub.shape))]
    got = got.cpu().numpy()
    assert np.isfinite(got).all()
    assert rel_err(got, want) <= FLOAT_TOL


@pytest.mark.parametrize("r", [1, 2])
def test_guided4d_tmarch_strided_view(r):
    """An in-place strided f32 view (row stride > nx, plane stride > ny * row stride) through the
    t-march and the buffer-access box3_final: the offsets built from the global (y, x) and the
    plane stride against the oracle of the same values made contiguous."""
    import torch
    rng = np.random.default_rng(60 + r)
    big = (rng.random((9, 14, 23, 77), dtype=np.float32) * 300).astype(np.float32)
    x = torch.from_numpy(big).cuda()[:, :, 1:-1, 2:-2]
    assert not x.is_contiguous() and x.stride()[2] > x.shape[3]
    v = np.ascontiguousarray(big[:, :, 1:-1, 2:-2])
    chunk = (3, 7, 7, 25)
    ref = O.guided_filter_apply(v, chunk, 0.5, r, nthreads=8)
    got = zt.GuidedFilter(0.5, r).apply_ndarray(x).cpu().numpy()
    assert rel_err(got, ref) <= FLOAT_TOL


# ---- 4-D one-march kernel (g4_fused.hip): T <= 4 timepoints per block, r <= 2 ---------------

@pytest.mark.parametrize("shape,chunk,r", [
    ((4, 40, 37, 150), (2, 16, 16, 64), 2),
    ((3, 70, 20, 65), (3, 32, 8, 32), 2),
    ((1, 33, 9, 130), (1, 8, 8, 64), 1),
    ((2, 45, 26, 71), (1, 16, 13, 40), 1),
    ((4, 12, 5, 7), (4, 4, 4, 4), 2),
])
def test_guided4d_fused_vs_oracle_small_eps(shape, chunk, r):
    rng = np.random.default_rng(sum(shape) + r)
    v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
    ref = O.guided_filter_apply(v, chunk, 0.5, r, nthreads=8)
    assert rel_err(gpu_apply(v, "float32", "float32", chunk, 0.5, r), ref) <= FLOAT_TOL
    assert rel_err(gpu_apply_chunked(v, "float32", "float32", chunk, 0.5, r), ref) <= FLOAT_TOL


# quad stage-1 loads (g4_fused_kernel<.., Q4>): r = 2, x extent a multiple of 4, several x tiles
# (the last one partial), fewer than 4 timepoints (the waves of timepoint 3 read zero-record
# descriptors), partial y tiles
@pytest.mark.parametrize("shape", [(3, 20, 21, 136), (4, 11, 9, 200), (2, 9, 40, 68)])
def test_guided4d_fused_quad_loads_vs_oracle(shape):
    rng = np.random.default_rng(sum(shape))
    v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
    chunk = (shape[0], 8, 8, 64)
    ref = O.guided_filter_apply(v, chunk, 0.5, 2, nthreads=8)
    assert rel_err(gpu_apply(v, "float32", "float32", chunk, 0.5, 2), ref) <= FLOAT_TOL


@pytest.mark.parametrize("din,dout", [("uint16", "float32"), ("float32", "uint8"),
                                      ("float64", "float16")])
def test_guided4d_fused_element_types(din, dout):
    rng = np.random.default_rng(43)
    v32 = (rng.random((4, 20, 17, 70), dtype=np.float32) * 200).astype(np.float32)
    v = O.cast_from_f32(v32, din)
    chunk = (2, 8, 8, 32)
    ref = O.guided_filter_apply(O.cast_to_f32(v, din), chunk, 300.0, 2, nthreads=8)
    check_against(gpu_apply(v, din, dout, chunk, 300.0, 2), ref, dout)


def test_guided4d_fused_chunk_grid_subset():
    import torch
    v = O.synth_step_noise_f32((4, 24, 16, 96))
    chunk = (2, 8, 8, 32)
    ref = O.guided_filter_apply(v, chunk, 2500.0, 2, nthreads=8)
    x = to_dev(v, "float32")
    y = torch.full(v.shape, -1.0, device="cuda")
    zt.GuidedFilter(2500.0, 2).apply(zt.DeviceArray(x, chunk), zt.DeviceArray(y, chunk),
                                     chunk_grid_start=(1, 1, 0, 1),
                                     chunk_grid_count=(1, 2, 1, 2))
    out = from_dev(y, "float32")
    box = (slice(2, 4), slice(8, 24), slice(0, 8), slice(32, 96))
    assert rel_err(out[box], ref[box]) <= FLOAT_TOL
    mask = np.ones(v.shape, bool)
    mask[box] = False
    assert np.all(out[mask] == -1)


# Launch grouping of the separable / four-kernel 4-D paths: with a scratch budget too small for
# the whole box (ZT_SCRATCH_LIMIT), chunks are grouped into rows over the trailing axes (or run
# one by one); every grouping equals the oracle. Each budget runs in its own process (the
# library reads the variable per call, torch state stays out of the parent).
@pytest.mark.parametrize("case", ["4d_rows", "4d_chunks", "3d_rows"])
def test_chunk_row_grouping_under_a_scratch_budget(case):
    import subprocess
    import sys
    code = f"""
import numpy as np, torch, sys
sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r})
from oracle import oracle as O
from tests.test_guided_filter_gpu import gpu_apply
from tests.gpu_util import rel_err, FLOAT_TOL
case = {case!r}
rng = np.random.default_rng(5)
if case.startswith("4d"):
    shape, chunk, r = (6, 40, 30, 70), (2, 8, 8, 32), 2
else:
    shape, chunk, r = (60, 40, 70), (8, 8, 32), 9
v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
ref = O.guided_filter_apply(v, chunk, 0.5, r, nthreads=8)
out = gpu_apply(v, "float32", "float32", chunk, 0.5, r)
e = rel_err(out, ref)
assert e <= FLOAT_TOL, e
print("ok", e)
"""
    # budgets: 4d_rows fits one (t, z) row of chunks (+ halo) but not the whole box; 4d_chunks
    # fits one chunk only; 3d_rows fits one z row of the separable path
    # (four-kernel scratch 20 B per input voxel, separable 5 f32 words; whole boxes 10.1 / 3.4 MB)
    limit = {"4d_rows": 20 * 6 * 16 * 30 * 70 + 64, "4d_chunks": 20 * 6 * 16 * 16 * 40 + 64,
             "3d_rows": 20 * 44 * 40 * 70 + 64}[case]
    env = dict(os.environ, ZT_SCRATCH_LIMIT=str(limit))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0 and "ok" in p.stdout, p.stderr[-2000:]
