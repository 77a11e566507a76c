"""CPU, multi-process (gloo, world_size 2 and 3): the per-GPU split of the chunk work queue used by
bench.py for N > 1 (zarrs_tools_amd.shard.slab_assignment). Each rank filters only its z-slab
plus the 2r halo rows (with the oracle, standing in for the device kernel), results are gathered
over gloo, and the union must equal the whole-volume filter. No data-path collective exists in
the real path; the gather here is only the test's checker. The max-over-ranks timing reduction
of bench.py is exercised the same way (all_reduce MAX)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from zarrs_tools_amd.shard import slab_assignment

SHAPE = (40, 12, 14)
CHUNK = 8
R = 2
EPS = 2500.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a = slab_assignment(rank, world, SHAPE[0], CHUNK, 2 * R)
        # the slab of the global synthetic volume this rank would generate on its device
        slab = O.synth_step_noise_f32((a.in_nz,) + SHAPE[1:], global_shape=SHAPE, z0=a.in_z0)
        res = O.guided_filter_apply_ndarray(slab, EPS, R)
        mine = np.zeros(SHAPE, np.float32)
        lo = a.out_z0 - a.in_z0
        mine[a.out_z0:a.out_z0 + a.out_nz] = res[lo:lo + a.out_nz]
        t = torch.from_numpy(mine)
        gathered = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(gathered, t)
        owned = torch.tensor([a.out_nz], dtype=torch.int64)
        dist.all_reduce(owned)                      # every row owned exactly once
        tmax = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks timing
        if rank == 0:
            q.put((sum(g.numpy() for g in gathered), int(owned), float(tmax)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_slab_split_with_halo_equals_whole_volume(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, owned, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert owned == SHAPE[0]
    assert tmax == float(world)
    whole = O.guided_filter_apply(O.synth_step_noise_f32(SHAPE), (CHUNK,) * 3, EPS, R, nthreads=4)
    assert np.abs(got - whole).max() <= 1e-5 * np.abs(whole).max()


def test_slab_assignment_covers_rows_once():
    for n_rows, chunk, world in [(2048, 256, 8), (100, 16, 3), (10, 16, 4), (64, 8, 5)]:
        seen = np.zeros(n_rows, int)
        for r in range(world):
            a = slab_assignment(r, world, n_rows, chunk, 8)
            seen[a.out_z0:a.out_z0 + a.out_nz] += 1
            assert a.in_z0 <= a.out_z0 and a.out_z0 + a.out_nz <= a.in_z0 + a.in_nz
            if a.out_nz:
                assert a.out_z0 % chunk == 0  # whole chunk rows per rank
                assert a.in_z0 == max(a.out_z0 - 8, 0)
                assert a.in_z0 + a.in_nz == min(a.out_z0 + a.out_nz + 8, n_rows)
        assert (seen == 1).all()


# ---- zarrs_ome pyramid: octant ownership (shard.octant_assignment) ---------------------------

from zarrs_tools_amd.shard import assemble_chunk, octant_assignment, pyramid_level_shapes  # noqa: E402


def _oracle_levels(v, factor, n):
    out, cur = [], v
    for _ in range(n):
        cur = O.downsample(cur, "uint16", factor, "uint16")
        out.append(cur)
    return out


def _octant_union(shape, factor, max_levels, world, gen):
    """Every rank's locally computed levels (the oracle standing in for the device kernel),
    assembled on the host level by level; levels past local_levels by rank 0 from the assembled
    level local_levels. Returns the assembled pyramid."""
    v = gen(shape)
    per_rank = []
    for r in range(world):
        a = octant_assignment(r, world, shape, factor, max_levels)
        if a.coord is None:
            per_rank.append((a, []))
            continue
        box = v[tuple(slice(s, s + n) for s, n in zip(a.start, a.shape))]
        per_rank.append((a, _oracle_levels(box, factor, a.local_levels)))
    a0 = per_rank[0][0]
    shapes = pyramid_level_shapes(shape, factor, max_levels)
    assert a0.levels == len(shapes)
    assembled = []
    for k in range(a0.local_levels):
        pieces = [(a.level_boxes[k][0], lv[k]) for a, lv in per_rank if a.coord is not None]
        for a, lv in per_rank:
            if a.coord is not None:
                assert lv[k].shape == a.level_boxes[k][1]
        assembled.append(assemble_chunk((0,) * len(shape), shapes[k], pieces))
    if a0.levels > a0.local_levels:
        assembled += _oracle_levels(assembled[-1], factor, a0.levels - a0.local_levels)
    return v, assembled


@pytest.mark.parametrize("shape,factor,world", [
    ((64, 48, 80), (2, 2, 2), 8), ((64, 48, 80), (2, 2, 2), 2), ((50, 37, 70), (2, 2, 2), 2),
    ((50, 37, 70), (2, 2, 2), 8), ((3, 8, 12), (2, 2, 2), 8), ((40, 36, 70), (2, 1, 2), 4),
    ((96, 64), (2, 2), 3), ((17, 33, 65), (3, 2, 2), 6)])
def test_octant_union_equals_global_pyramid(shape, factor, world):
    v, got = _octant_union(shape, factor, 10, world, O.synth_u16)
    want = _oracle_levels(v, factor, len(pyramid_level_shapes(shape, factor, 10)))
    assert len(got) == len(want)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


def test_octant_boxes_cover_each_level_once():
    shape, factor = (4096, 4096, 4096), (2, 2, 2)
    for world in (1, 2, 4, 8):
        shapes = pyramid_level_shapes(shape, factor, 5)
        for k in range(5):
            vol = 0
            for r in range(world):
                a = octant_assignment(r, world, shape, factor, 5)
                assert a.local_levels == 5 and a.coord is not None
                vol += int(np.prod(a.level_boxes[k][1]))
            assert vol == int(np.prod(shapes[k]))
    # config P: every rank owns a 2048^3 octant, levels 1-5 local (1024^3 .. 64^3)
    a = octant_assignment(7, 8, shape, factor, 5)
    assert a.shape == (2048,) * 3 and a.level_boxes[-1] == ((64, 64, 64), (64, 64, 64))


def _octant_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shape, factor = (48, 40, 72), (2, 2, 2)
        a = octant_assignment(rank, world, shape, factor, 10)
        # this rank's box of the global synthetic volume, generated locally
        box = O.synth_block_nd(a.start, a.shape, shape, "uint16")
        mine = _oracle_levels(box, factor, a.local_levels)
        got = [None] * world
        dist.all_gather_object(got, (a.level_boxes, [m.tolist() for m in mine]))
        if rank == 0:
            shapes = pyramid_level_shapes(shape, factor, 10)
            levels = []
            for k in range(a.local_levels):
                pieces = [(lb[k][0], np.array(lv[k], dtype=np.uint16)) for lb, lv in got]
                levels.append(assemble_chunk((0, 0, 0), shapes[k], pieces))
            q.put(levels)
    finally:
        dist.destroy_process_group()


def test_octant_split_gloo_world2_equals_whole_pyramid():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_octant_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    levels = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _oracle_levels(O.synth_u16((48, 40, 72)), (2, 2, 2), len(levels))
    for g, w in zip(levels, want):
        np.testing.assert_array_equal(g, w)


# ---- world size 8: the two splits an 8-GPU node runs -------------------------------------------
SHAPE_T = (16, 32, 5, 6)     # (t, z, y, x): 8 t-chunks x 4 z-chunks (config T: 8 x 4)
CHUNK_T = (2, 8, 5, 6)
R_T = 1


def _tz_worker(rank, world, port, q):
    """Config T's (t, z) block split (shard.block_split / block_assignment, the split
    zarrs_filter --gpus 8 and bench.py's T-share leg use): this rank filters its halo'd input box
    on its output box only (the oracle standing in for the device path), the boxes are gathered
    over gloo (the test's checker; the real path has no collective)."""
    from zarrs_tools_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        groups = shard.block_split(world, SHAPE_T, CHUNK_T, 2 * R_T)
        a = shard.block_assignment(rank, world, SHAPE_T, CHUNK_T, 2 * R_T, groups)
        mine = np.zeros(SHAPE_T, np.float32)
        cover = np.zeros(SHAPE_T[:2], np.int64)
        if int(np.prod(a.out_shape)):
            blk = O.synth_block_nd(a.in_start, a.in_shape, SHAPE_T, "float32")
            res = O.guided_filter_apply_ndarray(blk, EPS, R_T)
            src = tuple(slice(o - i, o - i + s) for o, i, s in zip(a.out_start, a.in_start,
                                                                 a.out_shape))
            dst = tuple(slice(o, o + s) for o, s in zip(a.out_start, a.out_shape))
            mine[dst] = res[src]
            cover[dst[:2]] += 1
        t, c = torch.from_numpy(mine), torch.from_numpy(cover)
        dist.all_reduce(t)
        dist.all_reduce(c)
        if rank == 0:
            q.put((t.numpy(), c.numpy(), tuple(groups)))
    finally:
        dist.destroy_process_group()


def test_tz_block_split_world8_equals_whole_series():
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tz_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, cover, groups = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert groups == (2, 4)  # config T's split: 2 t-groups x 4 z-groups
    assert (cover == 1).all()
    whole = O.guided_filter_apply(O.synth_step_noise_f32(SHAPE_T), CHUNK_T, EPS, R_T, nthreads=4)
    assert np.abs(got - whole).max() <= 1e-5 * np.abs(whole).max()
