"""CPU, multi-process: the orchestration of `zarrs_ome --gpus N` (zarrs_ome.run_octants). Each of
N spawned processes owns a factor^L-aligned box of level 0 (shard.octant_assignment), computes its
levels, writes the output chunks inside its box and hands the pieces of boundary-crossing chunks
to the parent, which assembles and writes them. Here the per-level compute of
each process is the oracle's downsample (test-only stand-in for the device kernel; the GPU test
test_cli_gpu.py::test_zarrs_ome_gpus_split_equals_one_process runs the HIP path); the partition,
the chunk writes, the host assembly and the pending-metadata protocol are the product code."""
import json
import os
import shutil

import numpy as np
import pytest

from oracle import oracle as O
from zarrs_tools_amd import shard
from zarrs_tools_amd import store as S
from zarrs_tools_amd import zarrs_ome as ZO


def _level_u16_2x(x):
    """One 2x2x2 mean level of a uint16 box (downsample.rs:72-97), the oracle's restatement."""
    return O.downsample(np.asarray(x), "uint16", (2, 2, 2), "uint16")


@pytest.mark.parametrize("world,prespawn,shape", [
    (2, False, (64, 48, 80)), (3, False, (64, 48, 80)), (4, False, (64, 48, 80)),
    (2, True, (64, 48, 80)),
    # config P's split on an 8-GPU node: 8 octants (2 x 2 x 2 rank grid), warmed-up workers
    (8, True, (64, 64, 96))])
def test_octant_processes_assemble_the_global_pyramid(tmp_path, world, prespawn, shape):
    chunk, factor = (16, 16, 16), (2, 2, 2)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, chunk)
    S.write_array(tmp_path / "in.zarr", u)
    root = tmp_path / "ome"
    os.makedirs(root)
    shutil.copytree(tmp_path / "in.zarr", root / "0")
    level_shapes = shard.pyramid_level_shapes(shape, factor, 10)
    L = shard.octant_assignment(0, world, shape, factor, len(level_shapes)).local_levels
    assert L >= 2
    ZO.prepare_octant_levels(str(root), level_shapes, L)
    # prespawn: the pool zarrs_ome.run starts first (octant_pool, one warm-up task per process)
    pool = ZO.octant_pool(world, [0] * world) if prespawn else None
    try:
        done, st = ZO.run_octants(str(root), shape, factor, len(level_shapes), False, world,
                                  devices=[0] * world, log=lambda *a: None,
                                  compute=_level_u16_2x, pool=pool)
    finally:
        if pool is not None:
            pool.shutdown()
    assert done == L
    assert st["assembled_chunks"] > 0  # the upper levels cross box boundaries
    assert st["processes"] == world
    if world == 8:
        assert list(st["grid"]) == [2, 2, 2]
    want = u
    for k in range(1, L + 1):
        want = _level_u16_2x(want)
        # not finished yet: no zarr.json until the parent publishes the level
        assert not os.path.exists(root / str(k) / "zarr.json")
        assert os.path.exists(root / str(k) / ZO.PENDING)
        np.testing.assert_array_equal(S.read_array(root / str(k)), want)
        ZO._publish_metadata(str(root / str(k)))
        m = json.load(open(root / str(k) / "zarr.json"))
        assert m["shape"] == list(level_shapes[k - 1])
    # the scratch directory of the pieces is gone
    assert not [p for p in os.listdir(root) if p.startswith(".zt_octants_")]


def test_box_chunks_inner_box_and_touched_chunks():
    lo, hi, i0, i1 = ZO._box_chunks((8, 0), (24, 40), (16, 16), (32, 40))
    assert (lo, hi) == ([0, 0], [2, 3])
    assert (i0, i1) == ([16, 0], [32, 40])  # the array end counts as a chunk boundary


@pytest.mark.parametrize("nthreads", [1, 8])
def test_copy_tree_equals_copytree(tmp_path, nthreads):
    # level 0's threaded copy (zarrs_ome.copy_tree) gives the tree shutil.copytree gives
    src = tmp_path / "in.zarr"
    S.create_array(src, "uint16", (40, 40, 40), (8, 8, 8))
    S.write_array(src, np.arange(40 ** 3, dtype=np.uint16).reshape(40, 40, 40), (0, 0, 0))
    ZO.copy_tree(str(src), str(tmp_path / "a"), nthreads)
    shutil.copytree(src, tmp_path / "b")
    walk = lambda r: sorted((os.path.relpath(d, r), sorted(f)) for d, _, f in os.walk(r))
    assert walk(tmp_path / "a") == walk(tmp_path / "b")
    for d, _, files in os.walk(tmp_path / "b"):
        for f in files:
            rel = os.path.relpath(os.path.join(d, f), tmp_path / "b")
            assert open(tmp_path / "a" / rel, "rb").read() == open(tmp_path / "b" / rel, "rb").read()
    np.testing.assert_array_equal(S.read_array(tmp_path / "a"), S.read_array(src))
    with pytest.raises(FileExistsError):
        ZO.copy_tree(str(src), str(tmp_path / "a"), nthreads)


def test_row_spans_cut_at_the_chunk_grid():
    from zarrs_tools_amd.zarrs_filter import _row_spans
    assert _row_spans(0, 16, 8) == [(0, 8), (8, 16)]
    assert _row_spans(5, 20, 8) == [(5, 8), (8, 16), (16, 24), (24, 25)]
    assert _row_spans(31, 6, 8) == [(31, 32), (32, 37)]
    assert _row_spans(3, 0, 8) == []


def test_read_pieces_are_chunk_aligned_and_cover_the_box(monkeypatch):
    from zarrs_tools_amd.zarrs_filter import _read_pieces
    start, shape, chunk = (5, 3, 0), (40, 37, 30), (8, 8, 16)
    whole = _read_pieces(start, shape, chunk, 2)  # default 512 MiB: whole chunk rows
    assert [(a, b) for a, b, _, _ in whole] == [(5, 8), (8, 16), (16, 24), (24, 32), (32, 40),
                                                (40, 45)]
    assert all((ya, yb) == (3, 40) for _, _, ya, yb in whole)
    monkeypatch.setenv("ZT_READ_PIECE_KB", "1")
    small = _read_pieces(start, shape, chunk, 2)
    cover = np.zeros(shape[:2], dtype=int)
    for a, b, ya, yb in small:
        assert (ya % 8 == 0 or ya == 3) and (yb % 8 == 0 or yb == 40)  # chunk grid / box ends
        cover[a - 5:b - 5, ya - 3:yb - 3] += 1
    assert (cover == 1).all()
    assert _read_pieces((0,), (20,), (8,), 4) == [(0, 8, 0, 1), (8, 16, 0, 1), (16, 20, 0, 1)]
