"""GPU: the multi-GPU splits run rank by rank on one device through the real per-rank entry
points, the union compared bit for bit with the whole-array result.

* octant pyramid (zarrs_ome): each rank's level-0 box through zt.pyramid
  (zt_pyramid_downsample), levels past local_levels by rank 0 from the assembled level;
* z-slab guided filter (bench.py strong scaling): zt_guided_filter_apply_slab per rank.
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.gpu_util import from_dev, to_dev

pytestmark = pytest.mark.gpu

import zarrs_tools_amd as zt  # noqa: E402
from zarrs_tools_amd.shard import assemble_chunk, octant_assignment, pyramid_level_shapes  # noqa: E402


@pytest.mark.parametrize("shape,world", [((256, 192, 320), 8), ((50, 37, 70), 2),
                                         ((3, 8, 12), 8), ((96, 64, 130), 4)])
def test_octant_pyramid_union_equals_whole(shape, world):
    import torch
    factor = (2, 2, 2)
    v = O.synth_u16(shape)
    x = to_dev(v, "uint16")
    whole = [from_dev(t, "uint16") for t in zt.pyramid(x, factor, 10)]
    shapes = pyramid_level_shapes(shape, factor, 10)
    assert [w.shape for w in whole] == shapes
    per_rank = []
    for r in range(world):
        a = octant_assignment(r, world, shape, factor, 10)
        if a.coord is None:
            continue
        box = x[tuple(slice(s, s + n) for s, n in zip(a.start, a.shape))].contiguous()
        lv = zt.pyramid(box, factor, a.local_levels)
        torch.cuda.synchronize()
        assert len(lv) == a.local_levels
        per_rank.append((a, [from_dev(t, "uint16") for t in lv]))
    a0 = per_rank[0][0]
    got = [assemble_chunk((0,) * 3, shapes[k], [(a.level_boxes[k][0], lv[k])
                                                for a, lv in per_rank])
           for k in range(a0.local_levels)]
    if a0.levels > a0.local_levels:
        rest = zt.pyramid(to_dev(got[-1], "uint16"), factor, a0.levels - a0.local_levels)
        got += [from_dev(t, "uint16") for t in rest]
    assert len(got) == len(whole)
    for g, w in zip(got, whole):
        np.testing.assert_array_equal(g, w)


def test_slab_split_world8_equals_whole():
    import torch
    from zarrs_tools_amd import _abi
    from zarrs_tools_amd.filter import _ptr
    shape, chunk, r = (64, 40, 96), (8, 16, 32), 4
    v = O.synth_step_noise_f32(shape)
    x = to_dev(v, "float32")
    y = torch.empty_like(x)
    zt.GuidedFilter(2500.0, r).apply(zt.DeviceArray(x, chunk), zt.DeviceArray(y, chunk))
    whole = from_dev(y, "float32")
    res = np.empty_like(v)
    for rank in range(8):
        a = zt.slab_assignment(rank, 8, shape[0], chunk[0], 2 * r)
        out = torch.empty((a.out_nz,) + shape[1:], device="cuda")
        slab = x[a.in_z0:a.in_z0 + a.in_nz].contiguous()
        _abi.check(_abi.lib().zt_guided_filter_apply_slab(
            zt.default_context().handle, 11, _ptr(slab), 11, _ptr(out), _abi.i64_array(shape),
            a.in_z0, a.in_nz, a.out_z0, a.out_nz, _abi.i64_array(chunk), 2500.0, r))
        torch.cuda.synchronize()
        res[a.out_z0:a.out_z0 + a.out_nz] = from_dev(out, "float32")
    assert np.array_equal(res, whole)


def test_synth_box_matches_oracle_block():
    import torch
    for kind, gshape, start, shape in [("uint16", (40, 36, 70), (8, 4, 33), (16, 20, 30)),
                                       ("float32", (9, 13, 70), (2, 1, 30), (5, 12, 40)),
                                       ("float32", (4, 6, 8, 10), (1, 2, 3, 4), (3, 4, 5, 6))]:
        d = zt.synth_box(start, shape, gshape, kind)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(from_dev(d, kind), O.synth_block_nd(start, shape, gshape, kind))
