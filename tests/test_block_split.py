"""(t, z) block partition of a 4-D chunk grid over ranks (shard.block_split / block_assignment,
config T): the ranks' output boxes tile the array with whole chunks, each input
box is its output box plus the 2r halo clamped to the array (ArraySubsetOverlap on the box), the
split minimises the input read in all, and filtering each rank's input box on its output box
reproduces the whole-array result (the oracle, CPU)."""
import itertools

import numpy as np
import pytest

from oracle import oracle as O
from zarrs_tools_amd import shard


@pytest.mark.parametrize("world,shape,chunk,halo", [
    (8, (32, 1024, 1024, 1024), (4, 256, 256, 256), 4),
    (4, (10, 14, 6, 5), (2, 3, 6, 5), 2),
    (6, (9, 20, 4, 4), (2, 4, 4, 4), 2),
    (3, (5, 5, 3, 3), (2, 2, 3, 3), 4),
])
def test_boxes_tile_the_array(world, shape, chunk, halo):
    g0, g1 = shard.block_split(world, shape, chunk, halo)
    assert g0 * g1 == world
    cover = np.zeros(shape[:2], np.int32)
    for r in range(world):
        a = shard.block_assignment(r, world, shape, chunk, halo)
        if int(np.prod(a.out_shape)) == 0:
            continue
        assert a.out_shape[2:] == tuple(shape[2:])
        for d in (0, 1):  # whole chunks (or the array end)
            assert a.out_start[d] % chunk[d] == 0
            end = a.out_start[d] + a.out_shape[d]
            assert end % chunk[d] == 0 or end == shape[d]
            assert a.in_start[d] == max(a.out_start[d] - halo, 0)
            assert a.in_start[d] + a.in_shape[d] == min(end + halo, shape[d])
        cover[a.out_start[0]:a.out_start[0] + a.out_shape[0],
              a.out_start[1]:a.out_start[1] + a.out_shape[1]] += 1
    assert (cover == 1).all()


def test_config_t_split_reads_less_than_rows_along_t():
    shape, chunk, halo = (32, 1024, 1024, 1024), (4, 256, 256, 256), 4

    def total(groups):
        return sum(int(np.prod(shard.block_assignment(r, 8, shape, chunk, halo, groups).in_shape))
                   for r in range(8))
    best = shard.block_split(8, shape, chunk, halo)
    assert best == (2, 4)
    rows = total((8, 1))
    assert total(best) < total((4, 2)) < rows
    out = int(np.prod(shape))
    assert rows / out == pytest.approx(2.75, rel=1e-3)      # 12 timepoints per 4 (edges: 8)
    assert total(best) / out == pytest.approx(1.27, rel=0.01)


@pytest.mark.parametrize("groups", [(2, 2), (4, 1), (1, 4)])
def test_blocks_equal_whole_array(groups):
    shape, chunk, radius = (8, 12, 6, 7), (2, 3, 6, 7), 1
    v = O.synth_step_noise_f32(shape)
    whole = O.guided_filter_apply_ndarray(v, 2500.0, radius)
    got = np.full(shape, np.nan, np.float32)
    for r in range(groups[0] * groups[1]):
        a = shard.block_assignment(r, 4, shape, chunk, 2 * radius, groups)
        blk = v[tuple(slice(s, s + n) for s, n in zip(a.in_start, a.in_shape))]
        res = O.guided_filter_apply_ndarray(np.ascontiguousarray(blk), 2500.0, radius)
        rel = tuple(slice(o - i, o - i + n) for o, i, n in zip(a.out_start, a.in_start,
                                                              a.out_shape))
        got[tuple(slice(o, o + n) for o, n in zip(a.out_start, a.out_shape))] = res[rel]
    assert not np.isnan(got).any()
    assert np.abs(got - whole).max() <= 1e-5 * max(1.0, np.abs(whole).max())
