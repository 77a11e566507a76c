"""GPU parity at the BASELINE.json configurations' full sizes, on samples of chunks.

Each case runs the HIP path over the whole configured volume (device-resident, synthetic data of
SURVEY.md §8(d)) and compares a sample of output chunks — corner, edge, interior — with the
oracle's per-chunk computation (the reference's apply_chunk: the 2r-halo input subset clamped to
the array, apply_ndarray on it, the halo dropped; guided_filter.rs:75-114). Downsample levels are
compared bit-exactly with the oracle's downsample of the same input region (downsample.rs:72-97).

  G2  guided_filter r=2, 1024^3 f32, 256^3 chunks        (BASELINE configs[1])
  G3  guided_filter r=4, 2048^3 f32, 256^3 chunks        (configs[2], the metric)
  P   5-level 2x mean pyramid of a 2048^3 u16 per-GPU octant of configs[3]'s 4096^3; the same
      size in u8 / i8, mean and mode (the packed-byte kernel)
  T   one GPU's share of configs[4]: rank 5's (t, z) block of the (2, 4) split of (32, 1024^3)
      f32 (output t [16, 32) x z [256, 512) from its 20 x 264-plane halo'd input block,
      shard.block_assignment), chunks (4, 256^3), r=2
  2-D 32768 x 16384 f32 (planes of 2 GiB: routed off the 32-bit fused path)
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.gpu_util import FLOAT_TOL

pytestmark = pytest.mark.gpu

import zarrs_tools_amd as zt  # noqa: E402

EPS = 2500.0


@pytest.fixture(autouse=True)
def _free_device_memory():
    """These cases hold tens of GiB: hand the memory back after each one."""
    yield
    import torch
    torch.cuda.synchronize()
    zt.default_context().release_scratch()
    torch.cuda.empty_cache()


def _check_chunks(out_dev, gshape, chunk, r, coords, z_off=0):
    refs = O.guided_filter_synth_chunks(gshape, chunk, coords, EPS, r, nthreads=16)
    worst, exact, total = 0.0, 0, 0
    for (o0, osh, ref) in refs:
        sl = tuple(slice(a - (z_off if d == 0 else 0), a - (z_off if d == 0 else 0) + s)
                   for d, (a, s) in enumerate(zip(o0, osh)))
        got = out_dev[sl].cpu().numpy()
        d = np.abs(got.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref.astype(np.float64)))
        worst = max(worst, float(d.max()))
        exact += int(np.count_nonzero(got == ref))
        total += got.size
    print(f"{gshape} r={r}: {len(coords)} chunks, max rel err {worst:.3e}, "
          f"bit-exact {exact / total:.4f}")
    assert worst <= FLOAT_TOL


def _guided_full(shape, chunk, r, n_interior=2):
    import torch
    x = zt.synth_step_noise_f32(shape)
    y = torch.empty_like(x)
    zt.GuidedFilter(EPS, r).apply(zt.DeviceArray(x, chunk), zt.DeviceArray(y, chunk))
    torch.cuda.synchronize()
    del x
    grid = [-(-s // c) for s, c in zip(shape, chunk)]
    _check_chunks(y, shape, chunk, r, O.sample_chunk_coords(grid, n_interior))


def test_g2_1024_r2_sampled_chunks():
    _guided_full((1024,) * 3, (256,) * 3, 2)


def test_g3_2048_r4_sampled_chunks():
    _guided_full((2048,) * 3, (256,) * 3, 4)


def test_g3_slab_split_sampled_chunks():
    """The strong-scaled bench form: each of 8 ranks' slabs (chunk row + 2r halo), run in turn on
    this GPU, checked on a chunk of its own row (the union covers every row once)."""
    import torch
    from zarrs_tools_amd import _abi
    from zarrs_tools_amd.filter import _ptr
    gshape, chunk, r = (2048, 2048, 2048), (256,) * 3, 4
    L = _abi.lib()
    ctx = zt.default_context()
    for rank in (0, 3, 7):
        a = zt.slab_assignment(rank, 8, gshape[0], 256, 2 * r)
        slab = torch.empty((a.in_nz,) + gshape[1:], dtype=torch.float32, device="cuda")
        out = torch.empty((a.out_nz,) + gshape[1:], dtype=torch.float32, device="cuda")
        _abi.check(L.zt_synth_step_noise_f32(ctx.handle, _ptr(slab), _abi.i64_array(slab.shape),
                                             3, _abi.i64_array(gshape), a.in_z0, O.SEED))
        _abi.check(L.zt_guided_filter_apply_slab(
            ctx.handle, 11, _ptr(slab), 11, _ptr(out), _abi.i64_array(gshape), a.in_z0, a.in_nz,
            a.out_z0, a.out_nz, _abi.i64_array(chunk), EPS, r))
        torch.cuda.synchronize()
        row = a.out_z0 // 256
        _check_chunks(out, gshape, chunk, r, [(row, 0, 7), (row, 4, 3)], z_off=a.out_z0)
        del slab, out


def test_p_pyramid_2048_u16_levels_bit_exact():
    import torch
    shape = (2048,) * 3
    x = zt.synth_u16(shape)
    levels = zt.pyramid(x, (2, 2, 2), max_levels=5)
    torch.cuda.synchronize()
    assert [tuple(t.shape) for t in levels] == [(1024,) * 3, (512,) * 3, (256,) * 3, (128,) * 3,
                                              (64,) * 3]
    # level 1: sampled 128^3 output boxes from the synthetic input (corner, interior, far corner)
    for o in [(0, 0, 0), (448, 320, 576), (896, 896, 896)]:
        src = O.synth_block_nd([2 * c for c in o], (256,) * 3, shape, "uint16")
        want = O.downsample(src, "uint16", (2, 2, 2), "uint16")
        got = levels[0][o[0]:o[0] + 128, o[1]:o[1] + 128, o[2]:o[2] + 128].cpu().numpy()
        np.testing.assert_array_equal(got, want)
    # levels 2..5: each from the GPU's previous level, whole level (<= 512^3 -> 256^3)
    for k in range(1, 5):
        prev = levels[k - 1]
        if prev.shape[0] > 256:
            prev = prev[:256, :256, :256]
        want = O.downsample(prev.cpu().numpy(), "uint16", (2, 2, 2), "uint16")
        got = levels[k][:want.shape[0], :want.shape[1], :want.shape[2]].cpu().numpy()
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("dtype,discrete", [("uint8", False), ("uint8", True),
                                             ("int8", False), ("int8", True)])
def test_pyramid_2048_bytes_levels_bit_exact(dtype, discrete):
    """The packed-byte pyramid kernel (pyramid3_u8_kernel: 16-byte rows, dot4 means, packed 16-bit
    sorting-network mode) at config P's per-GPU size: 5 levels of a 2048^3 u8 / i8 volume (the
    low byte of the synthetic u16; for the mode its low 3 bits, so majorities and ties occur)."""
    import torch
    shape = (2048,) * 3
    mask = 0x7 if discrete else 0xFF
    tt = torch.uint8 if dtype == "uint8" else torch.int8
    x = (zt.synth_u16(shape).view(torch.int16) & mask).to(tt)
    torch.cuda.synchronize()
    levels = zt.pyramid(x, (2, 2, 2), max_levels=5, discrete=discrete)
    torch.cuda.synchronize()
    del x
    for o in [(0, 0, 0), (448, 320, 576), (896, 896, 896)]:
        src = O.synth_block_nd([2 * c for c in o], (256,) * 3, shape, "uint16")
        src = (src & mask).astype(np.uint8).view(np.dtype(dtype))
        want = O.downsample(src, dtype, (2, 2, 2), dtype, discrete=discrete)
        got = levels[0][o[0]:o[0] + 128, o[1]:o[1] + 128, o[2]:o[2] + 128].cpu().numpy()
        np.testing.assert_array_equal(got, want)
    for k in range(1, 5):
        prev = levels[k - 1]
        if prev.shape[0] > 256:
            prev = prev[:256, :256, :256]
        want = O.downsample(prev.cpu().numpy(), dtype, (2, 2, 2), dtype, discrete=discrete)
        got = levels[k][:want.shape[0], :want.shape[1], :want.shape[2]].cpu().numpy()
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("rank", [5, 0])
def test_t_share_4d_sampled_chunks(rank):
    """Config T's real per-GPU share in the (t, z) block split of 8 GPUs
    (shard.block_assignment, 2 t-groups x 4 z-rows): rank 5 owns output timepoints [16, 32) x
    planes [256, 512) of the (32, 1024^3) series and holds its halo'd input block, timepoints
    [12, 32) x planes [252, 516), generated from the global synthetic definition (zt_synth_box).
    Every window clamps at the global array, which inside this block is the block's own bounds
    on the cut axes (the halo is complete), so apply_ndarray on the block's output box equals the
    reference's per-chunk result of the global array on sampled chunks (corner of the box, its
    last chunk, an interior one). Rank 0's block (output t [0, 16) x z [0, 256), input t [0, 20)
    x z [0, 260)) starts at the array's own t = 0 and z = 0 bounds: its corner chunk checks the
    clamped windows there."""
    import torch
    from zarrs_tools_amd import shard
    gshape, chunk, r = (32, 1024, 1024, 1024), (4, 256, 256, 256), 2
    a = shard.block_assignment(rank, 8, gshape, chunk, 2 * r, (2, 4))
    if rank == 5:
        assert a.out_start == (16, 256, 0, 0) and a.in_shape == (20, 264, 1024, 1024)
    else:
        assert a.out_start == (0, 0, 0, 0) and a.in_shape == (20, 260, 1024, 1024)
    x = zt.synth_box(a.in_start, a.in_shape, gshape, kind="float32")
    sub = zt.ArraySubset(tuple(o - i for o, i in zip(a.out_start, a.in_start)), a.out_shape)
    y = zt.GuidedFilter(EPS, r).apply_ndarray(x, sub)
    torch.cuda.synchronize()
    del x
    coords = [(4, 1, 0, 0), (7, 1, 3, 3), (5, 1, 2, 1)] if rank == 5 else \
        [(0, 0, 0, 0), (3, 0, 3, 2)]
    refs = O.guided_filter_synth_chunks(gshape, chunk, coords, EPS, r, nthreads=16)
    worst = 0.0
    for (o0, osh, ref) in refs:
        sl = tuple(slice(p - q, p - q + n) for p, q, n in zip(o0, a.out_start, osh))
        got = y[sl].cpu().numpy()
        d = np.abs(got.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref.astype(np.float64)))
        worst = max(worst, float(d.max()))
    print(f"config T share (t, z) block of rank {rank}: max rel err {worst:.3e}")
    assert worst <= FLOAT_TOL


def test_2d_plane_of_2gib_routes_off_the_fused_path():
    import torch
    shape, chunk, r = (32768, 16384), (256, 256), 2
    x = zt.synth_step_noise_f32(shape)
    y = torch.empty_like(x)
    zt.GuidedFilter(EPS, r).apply(zt.DeviceArray(x, chunk), zt.DeviceArray(y, chunk))
    torch.cuda.synchronize()
    del x
    _check_chunks(y, shape, chunk, r, [(0, 0), (127, 63), (64, 31), (127, 0), (5, 40)])
