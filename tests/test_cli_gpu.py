"""GPU: the zarrs_filter / zarrs_ome commands end to end on Zarr V3 stores, checked against the
oracle. The first case is BASELINE.json configs[0] (guided_filter on a 128^3 f32 synthetic
volume in 64^3 chunks) through the command line."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.gpu_util import FLOAT_TOL, rel_err

pytestmark = pytest.mark.gpu

from zarrs_tools_amd import store as S  # noqa: E402
from zarrs_tools_amd import zarrs_filter as ZF  # noqa: E402
from zarrs_tools_amd import zarrs_ome as ZO  # noqa: E402


def test_config0_cli_guided_filter_128(tmp_path):
    shape, chunk = (128, 128, 128), (64, 64, 64)
    S.create_array(tmp_path / "in.zarr", "float32", shape, chunk)
    S.write_synth(tmp_path / "in.zarr")
    rc = ZF.main(["guided-filter", str(tmp_path / "in.zarr"), str(tmp_path / "out.zarr"),
                  "2500", "2"])
    assert rc == 0
    out = S.read_array(tmp_path / "out.zarr")
    ref = O.guided_filter_apply(O.synth_step_noise_f32(shape), chunk, 2500.0, 2, nthreads=8)
    assert rel_err(out, ref) <= FLOAT_TOL


def test_run_config_chain_guided_then_downsample(tmp_path):
    shape, chunk = (40, 44, 48), (16, 16, 16)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, chunk)
    S.write_array(tmp_path / "in.zarr", u)
    cfg = tmp_path / "run.json"
    cfg.write_text(json.dumps([
        {"filter": "guided_filter", "input": str(tmp_path / "in.zarr"), "output": "$gf",
         "epsilon": 40000.0, "radius": 2, "data_type": "float32"},
        {"filter": "downsample", "output": str(tmp_path / "ds.zarr"), "stride": [2, 2, 2]},
    ]))
    assert ZF.main([str(cfg), "--tmp", str(tmp_path)]) == 0
    gf = O.guided_filter_apply(u.astype(np.float32), chunk, 40000.0, 2, nthreads=8)
    want = O.downsample(gf, "float32", (2, 2, 2), "float32")
    got = S.read_array(tmp_path / "ds.zarr")
    # the downsample of the GPU's guided filter output: the guided tolerance carries through
    assert rel_err(got, want) <= FLOAT_TOL


def _chain_cfg(tmp_path, inp, final):
    return [
        {"filter": "guided_filter", "input": inp, "output": "$gf", "epsilon": 40000.0,
         "radius": 2, "data_type": "float32"},
        {"filter": "gaussian", "sigma": [1.0, 1.0, 1.0], "kernel_half_size": [2, 2, 2]},
        {"filter": "downsample", "output": final, "stride": [2, 2, 2], "data_type": "uint16",
         "chunk_shape": [8, 8, 8], "bytes_to_bytes_codecs": '[{"name": "gzip", '
                                                            '"configuration": {"level": 1}}]'},
    ]


def test_device_resident_chain_equals_store_path(tmp_path):
    """A chain linked by temporaries runs on HBM arrays (zarrs_filter.rs:338-381 run configs,
    DESIGN.md §7): same output bits and the same output array as the step-by-step store path."""
    shape, chunk = (40, 44, 48), (16, 16, 16)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, chunk)
    S.write_array(tmp_path / "in.zarr", u)
    dev_out, store_out = str(tmp_path / "dev.zarr"), str(tmp_path / "store.zarr")
    logs = []
    res = ZF.run(_chain_cfg(tmp_path, str(tmp_path / "in.zarr"), dev_out), tmp=str(tmp_path),
                 log=logs.append)
    assert len(res) == 3 and all(r.get("device_resident") for r in res), logs
    res = ZF.run(_chain_cfg(tmp_path, str(tmp_path / "in.zarr"), store_out), tmp=str(tmp_path),
                 log=logs.append, device_chain=False)
    assert not any(r.get("device_resident") for r in res)
    a, b = S.read_array(dev_out), S.read_array(store_out)
    assert a.dtype == np.uint16 and a.shape == (20, 22, 24)
    assert np.array_equal(a, b)
    ma, mb = S.open_array(dev_out).metadata, S.open_array(store_out).metadata
    # (unsharded, --chunk-shape is overridden by the input's chunk grid as in
    # get_array_builder_reencode; the gzip codec is applied)
    assert ma == mb and any(c["name"] == "gzip" for c in ma["codecs"])
    # the oracle's chain (the guided tolerance carries through the later steps)
    gf = O.guided_filter_apply(u.astype(np.float32), chunk, 40000.0, 2, nthreads=8)
    g = O.gaussian_apply(gf, chunk, [1.0] * 3, [2] * 3)
    want = O.downsample(g, "float32", (2, 2, 2), "float32")
    assert np.max(np.abs(a.astype(np.float64) - want.astype(np.float64).astype(np.uint16))) <= 1
    # no temporary survives
    assert sorted(os.listdir(tmp_path)) == ["dev.zarr", "in.zarr", "store.zarr"]


def test_named_temporary_read_twice_is_not_chained(tmp_path):
    shape, chunk = (24, 20, 36), (8, 8, 16)
    v = O.synth_step_noise_f32(shape)
    S.create_array(tmp_path / "in.zarr", "float32", shape, chunk)
    S.write_array(tmp_path / "in.zarr", v)
    steps = [
        {"filter": "guided_filter", "input": str(tmp_path / "in.zarr"), "output": "$a",
         "epsilon": 2500.0, "radius": 1},
        {"filter": "downsample", "input": "$a", "output": str(tmp_path / "d1.zarr"),
         "stride": [2, 2, 2]},
        {"filter": "gaussian", "input": "$a", "output": str(tmp_path / "g.zarr"),
         "sigma": [1.0, 1.0, 1.0], "kernel_half_size": [1, 1, 1]},
    ]
    assert ZF.plan_chains(steps) == []
    res = ZF.run(steps, tmp=str(tmp_path), log=lambda *a: None)
    assert not any(r.get("device_resident") for r in res)
    gf = O.guided_filter_apply(v, chunk, 2500.0, 1, nthreads=8)
    assert rel_err(S.read_array(tmp_path / "g.zarr"),
                   O.gaussian_apply(gf, chunk, [1.0] * 3, [1] * 3)) <= FLOAT_TOL


def test_zarrs_ome_levels_and_metadata(tmp_path):
    shape, chunk = (40, 36, 70), (16, 16, 32)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, chunk, S.codecs_json("gzip"))
    S.write_array(tmp_path / "in.zarr", u)
    res = ZO.run(str(tmp_path / "in.zarr"), str(tmp_path / "ome"), max_levels=10,
                 log=lambda *a: None)
    lvl, want = 0, u
    while os.path.exists(tmp_path / "ome" / str(lvl + 1)):
        lvl += 1
        want = O.downsample(want, "uint16", (2, 2, 2), "uint16")
        np.testing.assert_array_equal(S.read_array(tmp_path / "ome" / str(lvl)), want)
    # 40,36,70 -> 20,18,35 -> 10,9,17 -> 5,4,8 -> 2,2,4 -> 1,1,2 -> 1,1,1: stop (zarrs_ome.rs:731)
    assert lvl == res["levels"] == 6
    meta = json.load(open(tmp_path / "ome" / "zarr.json"))
    ms = meta["attributes"]["ome"]["multiscales"][0]
    assert [d["path"] for d in ms["datasets"]] == [str(i) for i in range(7)]
    assert ms["datasets"][1]["coordinateTransformations"][0]["scale"] == [2.0, 2.0, 2.0]
    # cumulative scale = product of input/output per level (zarrs_ome.rs:570-578): the z axis
    # goes 5 -> 2 at level 4 (factor 2), 2 -> 1 (2), 1 -> 1 (1); y 9 -> 4 at level 3 (factor 2)
    shapes = [shape, (20, 18, 35), (10, 9, 17), (5, 4, 8), (2, 2, 4), (1, 1, 2), (1, 1, 1)]
    sc = [1.0, 1.0, 1.0]
    for lv in range(1, 7):
        sc = [a * (i // o) for a, i, o in zip(sc, shapes[lv - 1], shapes[lv])]
        ct = ms["datasets"][lv]["coordinateTransformations"]
        assert ct[0]["scale"] == sc
        assert ct[1]["translation"] == [(a - 1.0) * 0.5 for a in sc]


def test_zarrs_ome_extent3_factor2_scale(tmp_path):
    # extent 3 at factor 2: output 1, real factor 3 (the reference writes 3, not 2)
    shape, chunk = (3, 8, 12), (2, 4, 4)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, chunk)
    S.write_array(tmp_path / "in.zarr", u)
    ZO.run(str(tmp_path / "in.zarr"), str(tmp_path / "ome"), max_levels=1, log=lambda *a: None)
    np.testing.assert_array_equal(S.read_array(tmp_path / "ome" / "1"),
                                  O.downsample(u, "uint16", (2, 2, 2), "uint16"))
    meta = json.load(open(tmp_path / "ome" / "zarr.json"))
    ct = meta["attributes"]["ome"]["multiscales"][0]["datasets"][1]["coordinateTransformations"]
    assert ct[0]["scale"] == [3.0, 2.0, 2.0]
    assert ct[1]["translation"] == [1.0, 0.5, 0.5]


def test_guided_filter_with_reencoding_args(tmp_path):
    # -d float32 -s 32,32,32 -c 16,16,16 --bytes-to-bytes-codecs gzip: a sharded gzip output
    shape, chunk = (40, 44, 48), (16, 16, 16)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, chunk)
    S.write_array(tmp_path / "in.zarr", u)
    rc = ZF.main(["guided-filter", str(tmp_path / "in.zarr"), str(tmp_path / "out.zarr"),
                  "40000", "2", "-d", "float32", "-s", "32,32,32", "-c", "16,16,16",
                  "--bytes-to-bytes-codecs", '[{"name": "gzip", "configuration": {"level": 1}}]',
                  "--dimension-names", "z,y,x"])
    assert rc == 0
    m = json.load(open(tmp_path / "out.zarr" / "zarr.json"))
    assert m["data_type"] == "float32" and m["dimension_names"] == ["z", "y", "x"]
    assert m["chunk_grid"]["configuration"]["chunk_shape"] == [32, 32, 32]
    assert m["codecs"][0]["name"] == "sharding_indexed"
    ref = O.guided_filter_apply(u.astype(np.float32), chunk, 40000.0, 2, nthreads=8)
    assert rel_err(S.read_array(tmp_path / "out.zarr"), ref) <= FLOAT_TOL


def test_zarrs_ome_sharded_levels_reencoded_level0_and_axes(tmp_path):
    shape = (40, 36, 70)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, (16, 16, 32))
    S.write_array(tmp_path / "in.zarr", u)
    rc = ZO.main([str(tmp_path / "in.zarr"), str(tmp_path / "ome"), "--max-levels", "3",
                  "-s", "32,32,64", "-c", "16,16,32", "--physical-units",
                  "micrometer,micrometer,micrometer", "--physical-size", "2,1,1",
                  "--group-attributes", '{"note": "x"}', "--name", "vol"])
    assert rc == 0
    m0 = json.load(open(tmp_path / "ome" / "0" / "zarr.json"))
    assert m0["codecs"][0]["name"] == "sharding_indexed"  # level 0 reencoded (zarrs_ome.rs:355)
    np.testing.assert_array_equal(S.read_array(tmp_path / "ome" / "0"), u)
    want = u
    for lv in (1, 2, 3):
        want = O.downsample(want, "uint16", (2, 2, 2), "uint16")
        np.testing.assert_array_equal(S.read_array(tmp_path / "ome" / str(lv)), want)
        m = json.load(open(tmp_path / "ome" / str(lv) / "zarr.json"))
        assert m["codecs"][0]["name"] == "sharding_indexed"
    g = json.load(open(tmp_path / "ome" / "zarr.json"))["attributes"]
    assert g["note"] == "x"
    ms = g["ome"]["multiscales"][0]
    assert ms["name"] == "vol" and ms["type"] == "average"
    assert ms["axes"][0] == {"name": "0", "type": "space", "unit": "micrometer"}
    assert ms["coordinateTransformations"] == [{"type": "scale", "scale": [2.0, 1.0, 1.0]}]


def test_store_progress_callback_counts_output_chunks(tmp_path):
    shape, chunk = (40, 44, 48), (16, 16, 16)
    S.create_array(tmp_path / "in.zarr", "float32", shape, chunk)
    S.write_synth(tmp_path / "in.zarr")
    seen = []
    S.set_progress_callback(seen.append)
    try:
        S.guided_filter(tmp_path / "in.zarr", tmp_path / "out.zarr", 2500.0, 2)
    finally:
        S.set_progress_callback(None)
    n = 3 * 3 * 3
    assert [p["step"] for p in seen] == list(range(1, n + 1))
    assert all(p["num_steps"] == n for p in seen)
    assert seen[-1]["read_s"] > 0 and seen[-1]["write_s"] > 0 and seen[-1]["process_s"] > 0


def test_store_single_buffered_under_a_small_memory_budget(tmp_path, monkeypatch):
    # calculate_chunk_limit analogue: too little host memory for overlap -> one row in flight,
    # same result
    shape, chunk = (64, 48, 64), (16, 48, 64)
    S.create_array(tmp_path / "in.zarr", "float32", shape, chunk)
    S.write_synth(tmp_path / "in.zarr")
    row = 16 * 48 * 64 * 4
    monkeypatch.setenv("ZT_STORE_HOST_MEMORY", str(int(4 * row / 0.8) + 1024))
    st = S.guided_filter(tmp_path / "in.zarr", tmp_path / "out.zarr", 2500.0, 2)
    assert st["double_buffered"] == 0 and st["rows_in_flight"] == 3
    ref = O.guided_filter_apply(O.synth_step_noise_f32(shape), chunk, 2500.0, 2, nthreads=8)
    assert rel_err(S.read_array(tmp_path / "out.zarr"), ref) <= FLOAT_TOL


@pytest.mark.parametrize("mode", ["mean", "discrete", "gaussian"])
def test_zarrs_ome_device_resident_equals_store_levels(tmp_path, mode):
    """Levels computed from the previous level in HBM equal the reference's loop (each level
    read back from the store), bit for bit, with the same level metadata."""
    shape, chunk = (36, 40, 52), (16, 16, 16)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, chunk)
    S.write_array(tmp_path / "in.zarr", u)
    kw = {"discrete": mode == "discrete"}
    if mode == "gaussian":
        kw.update(gaussian_sigma=[1.0, 1.0, 1.0], gaussian_kernel_half_size=[2, 2, 2])
    a = ZO.run(str(tmp_path / "in.zarr"), str(tmp_path / "dev"), log=lambda *x: None, **kw)
    b = ZO.run(str(tmp_path / "in.zarr"), str(tmp_path / "store"), log=lambda *x: None,
               device_resident=False, **kw)
    assert all(st.get("device_resident") for st in a["stats"])
    assert not any(st.get("device_resident") for st in b["stats"])
    assert a["levels"] == b["levels"] >= 4
    for lvl in range(a["levels"] + 1):
        pa, pb = tmp_path / "dev" / str(lvl), tmp_path / "store" / str(lvl)
        assert np.array_equal(S.read_array(pa), S.read_array(pb)), lvl
        assert S.open_array(pa).metadata == S.open_array(pb).metadata
    with open(tmp_path / "dev" / "zarr.json") as f, open(tmp_path / "store" / "zarr.json") as g:
        assert json.load(f) == json.load(g)


def test_store_step_split_over_processes_equals_one_process(tmp_path):
    """zarrs_filter --gpus N: each store step split by output chunk rows over N processes (one
    per GPU; rehearsed here with every process on device 0) gives the one-process output, and
    zarr.json is written once at the end."""
    shape, chunk = (12, 20, 24, 40), (4, 8, 8, 16)  # 4-D: rows along t (config T's split)
    v = O.synth_step_noise_f32(shape)
    S.create_array(tmp_path / "in.zarr", "float32", shape, chunk)
    S.write_array(tmp_path / "in.zarr", v)
    steps = lambda out: [  # noqa: E731
        {"filter": "guided_filter", "input": str(tmp_path / "in.zarr"), "output": "$g",
         "epsilon": 2500.0, "radius": 2},
        {"filter": "downsample", "input": "$g", "output": out, "stride": [1, 2, 2, 2]},
    ]
    one = ZF.run(steps(str(tmp_path / "one.zarr")), tmp=str(tmp_path), log=lambda *a: None,
                 device_chain=False)
    two = ZF.run(steps(str(tmp_path / "two.zarr")), tmp=str(tmp_path), log=lambda *a: None,
                 gpus=2, gpu_devices=[0, 0])
    assert all(st.get("processes") == 2 for st in two)
    assert np.array_equal(S.read_array(tmp_path / "one.zarr"), S.read_array(tmp_path / "two.zarr"))
    assert S.open_array(tmp_path / "one.zarr").metadata == S.open_array(tmp_path / "two.zarr").metadata
    gf = O.guided_filter_apply(v, chunk, 2500.0, 2, nthreads=8)
    want = O.downsample(gf, "float32", (1, 2, 2, 2), "float32")
    assert rel_err(S.read_array(tmp_path / "one.zarr"), want) <= FLOAT_TOL


@pytest.mark.parametrize("gpus,mode", [(2, "mean"), (4, "mean"), (3, "discrete"),
                                       (2, "gaussian"), (2, "mean_pieces")])
def test_zarrs_ome_gpus_split_equals_one_process(tmp_path, gpus, mode, monkeypatch):
    """zarrs_ome --gpus N (rehearsed with every process on device 0): octant-owned levels with
    host assembly of boundary chunks (mean / mode), or every level split by chunk rows
    (--gaussian-sigma), give the one-process levels, level metadata and group metadata bit for
    bit. mean_pieces: 1 KiB read pieces (ZT_READ_PIECE_KB=1, inherited by the spawned workers),
    so the torch-free workers' box reads take the pitched hipMemcpy2DAsync sub-row copies."""
    if mode == "mean_pieces":
        monkeypatch.setenv("ZT_READ_PIECE_KB", "1")
        mode = "mean"
    shape, chunk = (64, 48, 80), (16, 16, 16)
    u = O.synth_u16(shape)
    S.create_array(tmp_path / "in.zarr", "uint16", shape, chunk)
    S.write_array(tmp_path / "in.zarr", u)
    kw = {"discrete": mode == "discrete"}
    if mode == "gaussian":
        kw.update(gaussian_sigma=[1.0, 1.0, 1.0], gaussian_kernel_half_size=[2, 2, 2])
    a = ZO.run(str(tmp_path / "in.zarr"), str(tmp_path / "one"), log=lambda *x: None, **kw)
    b = ZO.run(str(tmp_path / "in.zarr"), str(tmp_path / "many"), log=lambda *x: None,
               gpus=gpus, gpu_devices=[0] * gpus, **kw)
    if mode != "gaussian":
        assert b["stats"][0]["processes"] == gpus and b["stats"][0]["assembled_chunks"] > 0
        # the octant workers run without torch (ZT_NO_TORCH=1, hiprt.py)
        assert not any(r.get("torch_loaded") for r in b["stats"][0]["per_rank"])
    assert a["levels"] == b["levels"] >= 5
    for lvl in range(a["levels"] + 1):
        pa, pb = tmp_path / "one" / str(lvl), tmp_path / "many" / str(lvl)
        assert not os.path.exists(pb / ZO.PENDING)
        assert np.array_equal(S.read_array(pa), S.read_array(pb)), lvl
        assert S.open_array(pa).metadata == S.open_array(pb).metadata
    with open(tmp_path / "one" / "zarr.json") as f, open(tmp_path / "many" / "zarr.json") as g:
        assert json.load(f) == json.load(g)


def _rust_as(x, dt):
    """Rust `as` from float to an integer type: NaN -> 0, truncation, saturation."""
    info = np.iinfo(dt)
    y = np.nan_to_num(np.trunc(x.astype(np.float64)), nan=0.0, posinf=info.max, neginf=info.min)
    return np.clip(y, info.min, info.max).astype(dt)


def test_zarrs_ome_level0_data_type_reencodes_with_as_casts(tmp_path):
    """zarrs_ome -d: level 0 is the input converted with Rust `as` (Reencode, reencode.rs:58-77,
    zarrs_ome.rs:355-363) and the pyramid is built from it."""
    shape, chunk = (20, 24, 28), (8, 8, 8)
    v = (O.synth_step_noise_f32(shape) - 100.0) * np.float32(0.6)  # below 0 and above 255
    v[0, 0, :3] = [np.nan, np.inf, -np.inf]
    S.create_array(tmp_path / "in.zarr", "float32", shape, chunk)
    S.write_array(tmp_path / "in.zarr", v)
    assert ZO.main([str(tmp_path / "in.zarr"), str(tmp_path / "ome"), "--max-levels", "2",
                    "-d", "uint8"]) == 0
    l0 = S.read_array(tmp_path / "ome" / "0")
    np.testing.assert_array_equal(l0, _rust_as(v, np.uint8))
    assert json.load(open(tmp_path / "ome" / "0" / "zarr.json"))["data_type"] == "uint8"
    np.testing.assert_array_equal(S.read_array(tmp_path / "ome" / "1"),
                                  O.downsample(l0, "uint8", (2, 2, 2), "uint8"))
    # u16 -> f32 -> i16: exact values, then saturating truncation
    S.create_array(tmp_path / "u.zarr", "uint16", shape, chunk)
    u = O.synth_u16(shape)
    S.write_array(tmp_path / "u.zarr", u)
    assert ZO.main([str(tmp_path / "u.zarr"), str(tmp_path / "ome2"), "--max-levels", "1",
                    "-d", "float32"]) == 0
    np.testing.assert_array_equal(S.read_array(tmp_path / "ome2" / "0"), u.astype(np.float32))


def test_reencode_cast_matrix_matches_rust_as():
    """zt_reencode_cast over integer / float pairs whose Rust `as` numpy restates exactly."""
    import torch
    from zarrs_tools_amd import filter as F
    rng = np.random.default_rng(3)
    f = (rng.standard_normal(4096) * 300.0).astype(np.float32)
    f[:4] = [np.nan, np.inf, -np.inf, -0.0]
    i64 = rng.integers(-2 ** 40, 2 ** 40, 4096, dtype=np.int64)
    dev = torch.device("cuda", 0)
    for dt in (np.int8, np.int16, np.int32, np.uint8, np.uint16, np.uint32):
        got = F.reencode_cast(torch.from_numpy(f).to(dev), np.dtype(dt).name).cpu().numpy()
        np.testing.assert_array_equal(got, _rust_as(f, dt))
        got = F.reencode_cast(torch.from_numpy(i64).to(dev), np.dtype(dt).name).cpu().numpy()
        np.testing.assert_array_equal(got, i64.astype(dt))  # integer `as`: wrapping
    got = F.reencode_cast(torch.from_numpy(i64).to(dev), "float32").cpu().numpy()
    np.testing.assert_array_equal(got, i64.astype(np.float32))
    got = F.reencode_cast(torch.from_numpy(f).to(dev), "float64").cpu().numpy()
    np.testing.assert_array_equal(got, f.astype(np.float64))
    got = F.reencode_cast(torch.from_numpy(f).to(dev), "float16").cpu().numpy()
    np.testing.assert_array_equal(got.view(np.uint16), f.astype(np.float16).view(np.uint16))


def test_device_chain_failure_leaves_no_finished_output(tmp_path, monkeypatch):
    """A failing step of a device-resident chain leaves the chain output without zarr.json
    (zarrs_filter.rs:297-313: metadata only once the filter has finished)."""
    from zarrs_tools_amd import filter as F
    shape, chunk = (32, 32, 32), (16, 16, 16)
    S.create_array(tmp_path / "in.zarr", "float32", shape, chunk)
    S.write_synth(tmp_path / "in.zarr")

    def boom(*a, **k):
        raise RuntimeError("injected failure")
    monkeypatch.setattr(F.Gaussian, "apply", boom)
    steps = [{"filter": "guided_filter", "input": str(tmp_path / "in.zarr"), "output": "$g",
              "epsilon": 2500.0, "radius": 2},
             {"filter": "gaussian", "output": str(tmp_path / "out.zarr"), "sigma": [1.0] * 3,
              "kernel_half_size": [2] * 3}]
    with pytest.raises(RuntimeError, match="injected"):
        ZF.run(steps, tmp=str(tmp_path), log=lambda *a: None)
    assert not os.path.exists(tmp_path / "out.zarr" / "zarr.json")


def test_chunk_limit_bounds_chunks_in_flight(tmp_path):
    """--chunk-limit caps the chunks held in flight and the host threads (guided_filter.rs:
    251-258), down to one slab and one output row; the output is unchanged."""
    shape, chunk = (64, 32, 32), (8, 16, 16)  # 4 chunks per row, 8 chunk rows
    S.create_array(tmp_path / "in.zarr", "float32", shape, chunk)
    S.write_synth(tmp_path / "in.zarr")
    free = S.guided_filter(tmp_path / "in.zarr", tmp_path / "a.zarr", 2500.0, 2)
    lim = S.guided_filter(tmp_path / "in.zarr", tmp_path / "b.zarr", 2500.0, 2, chunk_limit=20)
    one = S.guided_filter(tmp_path / "in.zarr", tmp_path / "c.zarr", 2500.0, 2, chunk_limit=1)
    # a slab needs 3 input rows (r=2 halo over 8-plane rows): 5 decoded rows + 2 output rows
    # free; within 20 chunks 3 rows + 2 output rows; the floor is 3 rows + 1 output row
    assert free["rows_in_flight"] * 4 + 8 > 20
    assert (lim["rows_in_flight"], lim["double_buffered"]) == (3, 1)
    assert lim["threads"] <= 20 and one["threads"] == 1
    assert (one["rows_in_flight"], one["double_buffered"]) == (3, 0)
    a = S.read_array(tmp_path / "a.zarr")
    assert np.array_equal(a, S.read_array(tmp_path / "b.zarr"))
    assert np.array_equal(a, S.read_array(tmp_path / "c.zarr"))


@pytest.mark.parametrize("groups", [(2, 2), (1, 3), (3, 1)])
def test_store_guided_filter_tz_blocks_equal_whole(tmp_path, groups):
    """zt_store_guided_filter_box: the output written block by block — (t, z) boxes of whole
    chunks (shard.block_assignment), each read with the 2r halo along t and z — equals the
    one-call store output bit for bit, and the oracle within the float tolerance."""
    from zarrs_tools_amd import shard
    shape, chunk = (10, 22, 12, 20), (4, 8, 12, 10)
    v = O.synth_step_noise_f32(shape)
    S.create_array(tmp_path / "in.zarr", "float32", shape, chunk)
    S.write_array(tmp_path / "in.zarr", v)
    S.guided_filter(tmp_path / "in.zarr", tmp_path / "whole.zarr", 2500.0, 2)
    S.create_output(tmp_path / "in.zarr", tmp_path / "blocks.zarr", None, shape, None)
    world = groups[0] * groups[1]
    nt, nz = -(-shape[0] // chunk[0]), -(-shape[1] // chunk[1])
    for r in range(world):
        a = shard.block_assignment(r, world, shape, chunk, 4, groups)
        rows = (a.out_start[0] // chunk[0], -(-(a.out_start[0] + a.out_shape[0]) // chunk[0]))
        cols = (a.out_start[1] // chunk[1], -(-(a.out_start[1] + a.out_shape[1]) // chunk[1]))
        assert rows[1] <= nt and cols[1] <= nz
        S.guided_filter(tmp_path / "in.zarr", tmp_path / "blocks.zarr", 2500.0, 2, rows=rows,
                        cols=cols, erase=False, finish=False)
    got = S.read_array(tmp_path / "blocks.zarr")
    assert np.array_equal(got, S.read_array(tmp_path / "whole.zarr"))
    want = O.guided_filter_apply(v, chunk, 2500.0, 2, nthreads=8)
    assert rel_err(got, want) <= FLOAT_TOL
