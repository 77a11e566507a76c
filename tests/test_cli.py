"""CPU: the zarrs_filter / zarrs_ome command-line surface (argument grammar, run configs, error
behaviour) without device work. The GPU runs of the same commands are in test_cli_gpu.py."""
import json

import numpy as np
import pytest

from zarrs_tools_amd import _abi
from zarrs_tools_amd import store as S
from zarrs_tools_amd import zarrs_filter as ZF
from zarrs_tools_amd import zarrs_ome as ZO


def test_guided_filter_subcommand_grammar():
    # zarrs_filter guided-filter IN OUT EPSILON RADIUS [--data-type T] (guided_filter.rs:25-33)
    a = ZF.build_parser().parse_args(["guided-filter", "in.zarr", "out.zarr", "40000", "3",
                                      "--data-type", "float32"])
    steps = ZF._steps_from_cli(a)
    assert steps == [{"filter": "guided_filter", "input": "in.zarr", "output": "out.zarr",
                      "epsilon": 40000.0, "radius": 3, "data_type": "float32",
                      "chunk_limit": None}]


def test_downsample_subcommand_grammar():
    a = ZF.build_parser().parse_args(["downsample", "i", "o", "2,2,1", "--discrete"])
    assert ZF._steps_from_cli(a)[0]["stride"] == [2, 2, 1]
    assert ZF._steps_from_cli(a)[0]["discrete"] is True


def test_off_path_filter_is_rejected(tmp_path):
    S.create_array(tmp_path / "in", "uint8", (4,), (4,))
    with pytest.raises(_abi.FilterError, match="outside the accelerated path"):
        ZF.run([{"filter": "gradient_magnitude", "input": str(tmp_path / "in"), "output": "x"}],
               log=lambda *a: None)


def test_gaussian_subcommand_grammar():
    a = ZF.build_parser().parse_args(["gaussian", "i", "o", "1.0,1.5,2", "3,4,6",
                                      "--data-type", "float32"])
    st = ZF._steps_from_cli(a)[0]
    assert st["filter"] == "gaussian" and st["sigma"] == [1.0, 1.5, 2.0]
    assert st["kernel_half_size"] == [3, 4, 6] and st["data_type"] == "float32"


def test_gaussian_needs_one_sigma_per_axis(tmp_path):
    S.create_array(tmp_path / "in", "uint8", (4, 4), (4, 4))
    with pytest.raises(_abi.InvalidParameters, match="one entry per axis"):
        ZF.run([{"filter": "gaussian", "input": str(tmp_path / "in"), "output": "x",
                 "sigma": [1.0], "kernel_half_size": [3]}], log=lambda *a: None)


def test_first_filter_needs_input():
    with pytest.raises(_abi.InvalidParameters):
        ZF.run([{"filter": "guided_filter", "epsilon": 1.0, "radius": 1}], log=lambda *a: None)


def test_exists_exit_refuses_existing_output(tmp_path):
    S.create_array(tmp_path / "in", "float32", (4, 4), (2, 2))
    S.create_array(tmp_path / "out", "float32", (4, 4), (2, 2))
    with pytest.raises(_abi.FilterError, match="already exists"):
        ZF.run([{"filter": "guided_filter", "input": str(tmp_path / "in"),
                 "output": str(tmp_path / "out"), "epsilon": 1.0, "radius": 1}], exists="exit",
               log=lambda *a: None)


def test_run_config_file_and_missing_args(tmp_path):
    S.create_array(tmp_path / "in", "float32", (4, 4), (2, 2))
    cfg = tmp_path / "run.json"
    cfg.write_text(json.dumps([{"filter": "guided_filter", "input": str(tmp_path / "in"),
                                "output": "$tmp"}]))
    assert ZF.main([str(cfg)]) == 1  # no epsilon / radius -> InvalidParameters, exit code 1


def test_ome_factor_rank_mismatch(tmp_path):
    S.create_array(tmp_path / "in", "uint16", (8, 8), (4, 4))
    with pytest.raises(_abi.InvalidParameters):
        ZO.run(str(tmp_path / "in"), str(tmp_path / "out"), factor=[2, 2, 2], log=lambda *a: None)


def test_ome_scale_is_input_over_output_shape():
    # zarrs_ome.rs:570-578: real factor = input / output (integer), accumulated in f32. Extent 3 at
    # factor 2 -> output 1, factor 3; extent 11 at factor 4 -> output 2, factor 5.
    s = ZO.level_scale([1.0, 1.0, 1.0], (3, 11, 8), (1, 2, 4))
    assert s == [3.0, 5.0, 2.0]
    assert ZO.level_translation(s) == [1.0, 2.0, 0.5]
    s2 = ZO.level_scale(s, (1, 2, 4), (1, 1, 2))
    assert s2 == [3.0, 10.0, 4.0]


def test_exists_erase_removes_stale_chunks_under_tmp(tmp_path, monkeypatch):
    # an output under the temp root is erased like any other (prefix test skipped it)
    out = tmp_path / "out"
    S.create_array(out, "float32", (4, 4), (2, 2))
    (out / "c").mkdir(exist_ok=True)
    (out / "c" / "stale").write_bytes(b"x")
    calls = []
    monkeypatch.setattr(S, "guided_filter", lambda *a, **k: calls.append(a) or (_ for _ in ()).throw(
        _abi.FilterError(_abi.ERR_OTHER, "stop")))
    S.create_array(tmp_path / "in", "float32", (4, 4), (2, 2))
    with pytest.raises(_abi.FilterError, match="stop"):
        ZF.run([{"filter": "guided_filter", "input": str(tmp_path / "in"), "output": str(out),
                 "epsilon": 1.0, "radius": 1}], tmp=str(tmp_path), log=lambda *a: None)
    assert calls and not (out / "c" / "stale").exists()


def test_reencoding_args_on_every_filter():
    # ZarrReencodingArgs flattened into the filter arguments (filter_common_arguments.rs:7-16)
    a = ZF.build_parser().parse_args([
        "guided-filter", "i", "o", "1", "2", "-d", "float32", "-f", "NaN", "-s", "256,256,256",
        "-c", "32,32,32", "--bytes-to-bytes-codecs", '[{"name": "gzip", "configuration": {"level": 5}}]',
        "--separator", ".", "--dimension-names", "z,y,x", "--attributes", '{"k": 1}'])
    st = ZF._steps_from_cli(a)[0]
    enc = ZF.encoding_of(st)
    assert enc == {"data_type": "float32", "fill_value": "NaN", "separator": ".",
                   "chunk_shape": [32, 32, 32], "shard_shape": [256, 256, 256],
                   "bytes_to_bytes_codecs": [{"name": "gzip", "configuration": {"level": 5}}],
                   "dimension_names": ["z", "y", "x"], "attributes": {"k": 1}}
    for sub in (["downsample", "i", "o", "2,2"], ["gaussian", "i", "o", "1,1", "3,3"]):
        a = ZF.build_parser().parse_args(sub + ["--shard-shape", "0,64", "--fill-value", "3"])
        assert ZF.encoding_of(ZF._steps_from_cli(a)[0]) == {"shard_shape": [0, 64],
                                                           "fill_value": 3}
    # run-config form: JSON strings or values
    assert ZF.encoding_of({"filter": "downsample", "chunk_shape": "8,8",
                           "attributes_append": '{"a": 2}'}) == {
        "chunk_shape": [8, 8], "attributes_append": {"a": 2}}
    assert ZF.encoding_of({"filter": "downsample"}) is None


def test_ome_cli_surface_and_helpers():
    a = ZO.build_parser().parse_args(["i", "o", "2,2,1", "--physical-size", "0.5,0.5,1",
                                      "--physical-units", "micrometer,second,channel",
                                      "--group-attributes", '{"g": 1}', "--exists", "overwrite",
                                      "-s", "64,64,64", "-c", "32,32,32"])
    assert a.factor == [2, 2, 1] and a.physical_size == [0.5, 0.5, 1.0]
    assert a.exists == "overwrite" and a.shard_shape == [64, 64, 64]
    assert a.gpu_devices is None
    b = ZO.build_parser().parse_args(["i", "o", "--gpus", "2", "--gpu-devices", "0,0"])
    assert b.gpus == 2 and b.gpu_devices == [0, 0]
    # units_to_axis (zarrs_ome.rs:390-432)
    assert ZO.axis_of("z", "micrometer") == {"name": "z", "type": "space", "unit": "micrometer"}
    assert ZO.axis_of("t", "second") == {"name": "t", "type": "time", "unit": "second"}
    assert ZO.axis_of("c", "channel") == {"name": "c", "type": "channel"}
    assert ZO.axis_of("q", "furlong") == {"name": "q", "unit": "furlong"}
    assert ZO.axis_of("0", None) == {"name": "0"}


def test_ome_level_encoding_rule(tmp_path):
    # zarrs_ome.rs:528-560
    S.create_array(tmp_path / "a", "uint16", (40, 36, 70), (16, 16, 32))
    assert ZO.level_encoding(S.open_array(tmp_path / "a"), (20, 18, 35)) == {
        "chunk_shape": [16, 16, 32]}
    assert ZO.level_encoding(S.open_array(tmp_path / "a"), (5, 4, 8)) == {"chunk_shape": [5, 4, 8]}
    S.create_array(tmp_path / "b", "uint16", (40, 36, 70), (32, 32, 32),
                   S.codecs_json(None, shard_inner=(8, 16, 16)))
    assert ZO.level_encoding(S.open_array(tmp_path / "b"), (20, 18, 35)) == {
        "shard_shape": [20, 18, 32], "chunk_shape": [8, 16, 16]}


def test_plan_chains_links_only_private_temporaries():
    from zarrs_tools_amd.zarrs_filter import plan_chains
    g = {"filter": "guided_filter", "epsilon": 1.0, "radius": 1}
    # implicit outputs / inputs chain; a named final output ends the chain
    steps = [dict(g, input="in"), dict(g), dict(g, output="out")]
    assert plan_chains(steps) == [(0, 2)]
    # "$t" written by 0 and read only by 1
    steps = [dict(g, input="in", output="$t"), dict(g, input="$t", output="out")]
    assert plan_chains(steps) == [(0, 1)]
    # "$t" read by two steps: no chain through it
    steps = [dict(g, input="in", output="$t"), dict(g, input="$t", output="o1"),
             dict(g, input="$t", output="o2")]
    assert plan_chains(steps) == []
    # a named (non-temporary) intermediate breaks the chain
    steps = [dict(g, input="in", output="mid"), dict(g, output="out")]
    assert plan_chains(steps) == []
    # two chains separated by a named output
    steps = [dict(g, input="in"), dict(g, output="m"), dict(g, input="m"), dict(g, output="o")]
    assert plan_chains(steps) == [(0, 1), (2, 3)]
