"""CPU: bench.py's host logic — the post-timing parity sample against the oracle, the
chunk-row split of the strong-scaled volume, and the --gpus / WORLD_SIZE launcher check."""
import numpy as np
import pytest
import torch

import bench
from oracle import oracle as O
import zarrs_tools_amd as zt


def test_parity_sample_matches_whole_volume_oracle(monkeypatch):
    monkeypatch.setattr(bench, "CHUNK", 16)
    gshape, r = (48, 32, 48), 2
    v = O.synth_step_noise_f32(gshape)
    whole = O.guided_filter_apply(v, (16, 16, 16), bench.EPS, r, nthreads=4)
    for rank in range(2):
        a = zt.slab_assignment(rank, 2, gshape[0], 16, 2 * r)
        out = torch.from_numpy(whole[a.out_z0:a.out_z0 + a.out_nz].copy())
        res = bench.parity_sample(out, a, gshape, r, 4)
        assert res["ok"] and res["max_rel"] == 0.0 and res["bit_exact_frac"] == 1.0
        assert all(a.out_z0 // 16 <= c[0] < (a.out_z0 + a.out_nz) // 16 for c in res["chunks"])
    # a corrupted voxel in a sampled chunk is caught
    a = zt.slab_assignment(0, 1, gshape[0], 16, 2 * r)
    bad = torch.from_numpy(whole.copy())
    bad[0, 0, 0] += 1.0
    assert not bench.parity_sample(bad, a, gshape, r, 4)["ok"]


def test_strong_split_covers_the_volume_once():
    for world in (1, 2, 4, 8):
        rows = []
        for g in range(world):
            a = zt.slab_assignment(g, world, 2048, 256, 8)
            rows += list(range(a.out_z0, a.out_z0 + a.out_nz))
            assert a.in_z0 == max(a.out_z0 - 8, 0)
            assert a.in_z0 + a.in_nz == min(a.out_z0 + a.out_nz + 8, 2048)
        assert rows == list(range(2048))


def test_gpus_must_match_world_size(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")

    class A:
        gpus = 4
    with pytest.raises(SystemExit) as e:
        bench.maybe_launch(A())
    assert e.value.code == 2
    A.gpus = 2
    bench.maybe_launch(A())  # under a launcher with the matching count: no-op


def test_traffic_entries_are_keyed_to_build_workload_and_world(monkeypatch, tmp_path):
    import json
    (tmp_path / "profiles").mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_hash", lambda: "abc")
    entries = [{"lib_sha256": "abc", "global_shape": [2048] * 3, "radius": 4, "world": 1,
                "hbm_bytes_per_launch": 1.0e11},
               {"lib_sha256": "abc", "global_shape": [1024] * 3, "radius": 2, "world": 1,
                "hbm_bytes_per_launch": 2.0e10},
               {"lib_sha256": "old", "global_shape": [512] * 3, "radius": 2, "world": 1,
                "hbm_bytes_per_launch": 3.0e9}]
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps({"entries": entries}))
    assert bench.load_traffic((2048,) * 3, 4, 1) == 1.0e11
    assert bench.load_traffic((1024,) * 3, 2, 1) == 2.0e10
    assert bench.load_traffic((512,) * 3, 2, 1) is None  # measured on another build
    assert bench.load_traffic((2048,) * 3, 4, 2) is None  # another world size
    # a --share G/N proxy line never carries the whole volume's traffic, only an
    # entry measured on that share
    assert bench.load_traffic((2048,) * 3, 4, 1, (3, 8)) is None
    shared = dict(entries[0], share=[3, 8], hbm_bytes_per_launch=1.9e10)
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(
        json.dumps({"entries": entries + [shared]}))
    assert bench.load_traffic((2048,) * 3, 4, 1, (3, 8)) == 1.9e10
    assert bench.load_traffic((2048,) * 3, 4, 1, (2, 8)) is None
    assert bench.load_traffic((2048,) * 3, 4, 1) == 1.0e11
    # the single-entry form of earlier rounds still reads
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(entries[0]))
    assert bench.load_traffic((2048,) * 3, 4, 1) == 1.0e11


def test_sq_counters_follow_the_traffic_key(monkeypatch, tmp_path):
    """The SQ instruction counters per voxel (report G2's SALU / voxel in its leg)
    ride on the same keyed PMC entry as the traffic: reported only for this build and workload."""
    import json
    (tmp_path / "profiles").mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_hash", lambda: "abc")
    sq = {"VALU": 0.85, "SALU": 0.42, "LDS": 0.18}
    entries = [{"lib_sha256": "abc", "global_shape": [1024] * 3, "radius": 2, "world": 1,
                "hbm_bytes_per_launch": 2.0e10, "sq_per_voxel": sq,
                "sq_wave_cycle_ratios": {"WAIT_INST_ANY": 0.36}},
               {"lib_sha256": "abc", "global_shape": [2048] * 3, "radius": 4, "world": 1,
                "hbm_bytes_per_launch": 1.0e11},
               {"lib_sha256": "old", "global_shape": [512] * 3, "radius": 2, "world": 1,
                "hbm_bytes_per_launch": 3.0e9, "sq_per_voxel": sq}]
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps({"entries": entries}))
    got = bench.load_sq((1024,) * 3, 2, 1)
    assert got["insts_per_voxel"] == sq and got["wave_cycle_ratios"] == {"WAIT_INST_ANY": 0.36}
    assert bench.load_sq((2048,) * 3, 4, 1) is None  # traffic only, no SQ passes
    assert bench.load_sq((512,) * 3, 2, 1) is None  # another build
    assert bench.load_traffic((1024,) * 3, 2, 1) == 2.0e10
