"""GPU: bench.py end to end as the driver runs it. `--gpus 2` starts its own two ranks through
torch.distributed.run (here rehearsed with both ranks on device 0 and a gloo barrier,
ZT_BENCH_ONE_DEVICE=1: the 8-GPU run is the driver's), and `--share G/N` times one rank's slab
of an N-way split alone (the per-rank proxy of the strong-scaling run). Each prints one JSON line
with the ranks, the max-over-ranks timing and the post-timing parity sample."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_launcher_rehearsal():
    r = _run(["--gpus", "2", "--size", "512", "--steps", "2", "--warmup", "1",
              "--parity-chunks", "3"], {"ZT_BENCH_ONE_DEVICE": "1"})
    assert r["ranks"] == 2 and r["n_gpus"] == 1  # two ranks sharing device 0
    assert r["scaling"] == "strong" and r["config"]["parallelism"] == "chunk-rows x2 (strong)"
    assert r["parity"]["ok"] and r["parity_max_rel"] <= 1e-5
    assert r["value"] > 0 and r["roofline"]["kernel_ms"] > 0
    assert "cpu_baseline" not in r  # N > 1 lines carry no CPU baseline


def test_bench_share_proxy_of_an_eight_way_split():
    r = _run(["--share", "3/8", "--size", "2048", "--steps", "2", "--warmup", "1",
              "--parity-chunks", "2", "--no-cpu-baseline"])
    assert r["share"]["rank"] == 3 and r["share"]["world"] == 8
    assert r["share"]["out_z"] == [768, 1024] and r["share"]["in_z"] == [760, 1032]
    assert r["parity"]["ok"]
    assert r["share"]["projected_aggregate_gibs"] == pytest.approx(r["value"] * 8, rel=1e-3)


def test_bench_rccl_process_group_at_one_rank():
    """The N-GPU path's RCCL calls (init_process_group("nccl", device_id=...), barrier, MAX
    all-reduce of the timings) on a 1-GPU box: one rank under torch.distributed.run with
    ZT_BENCH_DIST=1."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["ZT_BENCH_DIST"] = "1"
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=1", "--master-addr", "127.0.0.1",
                        f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--size", "512",
                        "--steps", "2", "--warmup", "1", "--parity-chunks", "2",
                        "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["dist_backend"] == "nccl" and r["ranks"] == 1
    assert r["parity"]["ok"] and r["value"] > 0
