"""CPU: the output array builder of the filters (FilterTraits::output_array_builder,
filter_traits.rs:47-82 + get_array_builder_reencode, lib.rs:408-650) through
zt_store_create_output_like, and the calculate_chunk_limit analogue of the store pipeline
(filter.rs:52-66). No device work: the memory check fails before the GPU is touched."""
import json

import pytest

from zarrs_tools_amd import _abi
from zarrs_tools_amd import store as S


def _meta(path):
    return json.load(open(path / "zarr.json"))


def _mk(tmp_path, sharded=False, **kw):
    codecs = S.codecs_json("gzip", shard_inner=(8, 8, 16)) if sharded else S.codecs_json("gzip")
    S.create_array(tmp_path / "in", "uint16", (40, 36, 70), (16, 16, 32), codecs, **kw)
    return tmp_path / "in"


def test_default_output_is_like_input(tmp_path):
    src = _mk(tmp_path)
    S.create_output_like(src, tmp_path / "out")
    a, b = _meta(src), _meta(tmp_path / "out")
    for k in ("shape", "data_type", "chunk_grid", "codecs", "fill_value", "chunk_key_encoding"):
        assert a[k] == b[k], k


def test_data_type_converts_fill_value(tmp_path):
    S.create_array(tmp_path / "in", "float32", (8, 8), (4, 4), fill_value=-3.7)
    S.create_output_like(tmp_path / "in", tmp_path / "o1", "uint8")
    m = _meta(tmp_path / "o1")
    assert m["data_type"] == "uint8" and m["fill_value"] == 0  # -3.7 as u8 saturates to 0
    S.create_output_like(tmp_path / "in", tmp_path / "o2", None,
                         {"data_type": "int16", "fill_value": 7})
    m = _meta(tmp_path / "o2")
    assert m["data_type"] == "int16" and m["fill_value"] == 7


def test_shard_shape_on_unsharded_input(tmp_path):
    src = _mk(tmp_path)
    S.create_output_like(src, tmp_path / "o", None, {"shard_shape": [32, 0, 40],
                                                     "chunk_shape": [16, 12, 16]})
    m = _meta(tmp_path / "o")
    # shard = min(s, extent) (0 = extent), rounded up to a multiple of the chunk (lib.rs:474-494)
    assert m["chunk_grid"]["configuration"]["chunk_shape"] == [32, 36, 48]
    sh = m["codecs"][0]
    assert sh["name"] == "sharding_indexed"
    assert sh["configuration"]["chunk_shape"] == [16, 12, 16]
    assert [c["name"] for c in sh["configuration"]["codecs"]] == ["bytes", "gzip"]
    assert [c["name"] for c in sh["configuration"]["index_codecs"]] == ["bytes", "crc32c"]
    # without a chunk shape the inner chunk is the input's chunk GRID shape (lib.rs:447)
    S.create_output_like(src, tmp_path / "o2", None, {"shard_shape": [16, 16, 32]})
    sh = _meta(tmp_path / "o2")["codecs"][0]["configuration"]
    assert sh["chunk_shape"] == [3, 3, 3]


def test_chunk_shape_alone_keeps_the_input_grid(tmp_path):
    # get_array_builder_reencode applies the chunk shape only with sharding (lib.rs:623-646)
    src = _mk(tmp_path)
    S.create_output_like(src, tmp_path / "o", None, {"chunk_shape": [8, 8, 8]})
    assert _meta(tmp_path / "o")["chunk_grid"] == _meta(src)["chunk_grid"]


def test_sharded_input_keeps_inner_chunks_and_codec_overrides(tmp_path):
    src = _mk(tmp_path, sharded=True)
    S.create_output_like(src, tmp_path / "o", None, {
        "bytes_to_bytes_codecs": [{"name": "crc32c"}], "separator": ".",
        "dimension_names": ["z", "y", "x"], "attributes": {"a": 1},
        "attributes_append": {"b": [2]}})
    m = _meta(tmp_path / "o")
    assert m["chunk_grid"]["configuration"]["chunk_shape"] == [16, 16, 32]
    cfg = m["codecs"][0]["configuration"]
    assert cfg["chunk_shape"] == [8, 8, 16]
    assert [c["name"] for c in cfg["codecs"]] == ["bytes", "crc32c"]
    assert m["chunk_key_encoding"] == {"name": "default", "configuration": {"separator": "."}}
    assert m["dimension_names"] == ["z", "y", "x"] and m["attributes"] == {"a": 1, "b": [2]}


def test_bad_encodings_are_rejected(tmp_path):
    src = _mk(tmp_path)
    with pytest.raises(_abi.InvalidParameters, match="unknown key"):
        S.create_output_like(src, tmp_path / "o", None, {"chunkshape": [1, 1, 1]})
    with pytest.raises(_abi.InvalidParameters, match="array to array"):
        S.create_output_like(src, tmp_path / "o", None, {
            "array_to_array_codecs": [{"name": "transpose", "configuration": {"order": [0, 2, 1]}}]})
    with pytest.raises(_abi.FilterError):
        S.create_output_like(src, tmp_path / "o", None, {"data_type": "complex64"})


def test_not_enough_memory_is_the_reference_error(tmp_path, monkeypatch):
    S.create_array(tmp_path / "in", "float32", (64, 64, 64), (32, 64, 64))
    monkeypatch.setenv("ZT_STORE_HOST_MEMORY", "100000")  # < one 512 KiB chunk row
    with pytest.raises(_abi.FilterError, match="not enough available memory") as e:
        S.guided_filter(tmp_path / "in", tmp_path / "out", 1.0, 1)
    assert e.value.status == _abi.ERR_OUT_OF_MEMORY
