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
