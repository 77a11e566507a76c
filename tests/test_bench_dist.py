"""CPU, multi-process (gloo): the agreement and timing helpers of bench.py's distributed legs
(configs[3] and [4] timed across the ranks when N > 1). A leg allocates and warms up on every
rank, then the ranks agree before any timed barrier: an error on one rank must make every rank
skip the leg (nobody left waiting at a barrier the others never reach), and the reported time is
the max over ranks. The device synchronisation is stubbed out (no GPU here); the legs' kernels
are covered by the GPU rehearsal (profiles/r06_rehearse_*ranks_one_gpu.json)."""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fail_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.synchronize = lambda *a, **k: None  # no device in this test
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []

        def prepare():
            if rank == fail_rank:
                raise MemoryError("out of memory on this rank")
            calls.append("prepare")

        def step():
            time.sleep(0.01 * (rank + 1))  # the slowest rank sets the time
            calls.append("step")

        err = bench._dist_prepare(prepare, step, dist, "cpu", True, 1)
        ms = None
        if err is None:
            ms = bench._dist_time(step, dist, "cpu", True, 0, 3)
        # a collective after the leg: every rank must still be in step with the others
        after = bench._dist_reduce([float(rank)], dist.ReduceOp.MAX, dist, "cpu", True)[0]
        q.put((rank, err, ms, after))
    finally:
        dist.destroy_process_group()


def _run(world, fail_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fail_rank, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_dist_leg_timing_is_max_over_ranks(world):
    res = _run(world, fail_rank=-1)
    for rank, err, ms, after in res:
        assert err is None
        assert after == world - 1
        # the slowest rank sleeps 10 * world ms per step; every rank reports that maximum
        assert ms >= 10.0 * world * 0.9
    assert len({round(r[2], 6) for r in res}) == 1


@pytest.mark.parametrize("world,fail_rank", [(2, 1), (3, 0)])
def test_dist_leg_error_on_one_rank_skips_everywhere(world, fail_rank):
    res = _run(world, fail_rank)
    for rank, err, ms, after in res:
        assert err is not None and ms is None
        if rank == fail_rank:
            assert "MemoryError" in err
        else:
            assert err == "failed on another rank"
        assert after == world - 1  # the ranks left the leg together
