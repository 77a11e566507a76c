"""CPU: the Zarr V3 filesystem store under the store -> store path (no device work).

The reference reads and writes these arrays through zarrs (Array::open / ArrayBuilder::build,
retrieve/store_array_subset_ndarray; src/bin/zarrs_filter.rs:63-87, guided_filter.rs:95-110).
Round trips through every supported codec chain, edge (partial) chunks, missing chunks = fill
value, sharding with a crc32c-checked index, and the synthetic generator against the oracle."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from zarrs_tools_amd import store as S
from zarrs_tools_amd import _abi

CHAINS = [
    ("bytes", dict()),
    ("gzip", dict(compression="gzip", level=1)),
    ("shard", dict(shard_inner=(4, 5, 8))),
    ("shard_gzip", dict(compression="gzip", level=5, shard_inner=(8, 5, 4))),
]
if S.codec_available("zstd"):
    CHAINS.append(("zstd", dict(compression="zstd", level=3)))


@pytest.mark.parametrize("name,kw", CHAINS, ids=[c[0] for c in CHAINS])
@pytest.mark.parametrize("dtype", ["float32", "uint16", "int8", "float64"])
def test_round_trip_codecs(tmp_path, name, kw, dtype):
    shape, chunk = (13, 17, 19), (8, 10, 16)  # partial edge chunks on every axis
    p = tmp_path / "a.zarr"
    S.create_array(p, dtype, shape, chunk, S.codecs_json(**kw))
    rng = np.random.default_rng(7)
    data = (rng.standard_normal(shape) * 50).astype(S.NUMPY[dtype])
    S.write_array(p, data)
    back = S.read_array(p)
    np.testing.assert_array_equal(back, data)
    # unaligned subset read spanning chunks
    sub = S.read_array(p, start=(3, 4, 5), shape=(9, 11, 12))
    np.testing.assert_array_equal(sub, data[3:12, 4:15, 5:17])
    meta = json.load(open(p / "zarr.json"))
    assert meta["zarr_format"] == 3 and meta["node_type"] == "array"
    assert meta["shape"] == list(shape) and meta["data_type"] == dtype
    assert meta["chunk_grid"]["configuration"]["chunk_shape"] == list(chunk)


def test_missing_chunks_read_fill_value(tmp_path):
    p = tmp_path / "f.zarr"
    S.create_array(p, "float32", (6, 6), (4, 4), fill_value=2.5)
    S.write_array(p, np.ones((4, 4), np.float32), start=(0, 0))
    back = S.read_array(p)
    want = np.full((6, 6), 2.5, np.float32)
    want[:4, :4] = 1
    np.testing.assert_array_equal(back, want)


def test_nan_fill_value_and_metadata(tmp_path):
    p = tmp_path / "n.zarr"
    S.create_array(p, "float32", (3,), (2,), fill_value="NaN")
    assert json.load(open(p / "zarr.json"))["fill_value"] == "NaN"
    assert np.isnan(S.read_array(p)).all()


def test_shard_index_crc_detects_corruption(tmp_path):
    p = tmp_path / "s.zarr"
    S.create_array(p, "uint16", (8, 8), (8, 8), S.codecs_json(shard_inner=(4, 4)))
    S.write_array(p, np.arange(64, dtype=np.uint16).reshape(8, 8))
    f = p / "c" / "0" / "0"
    raw = bytearray(f.read_bytes())
    raw[-6] ^= 0xFF  # inside the index
    f.write_bytes(bytes(raw))
    with pytest.raises(_abi.FilterError, match="crc32c"):
        S.read_array(p)


def test_chunk_key_encoding_default(tmp_path):
    p = tmp_path / "k.zarr"
    S.create_array(p, "uint8", (4, 4, 4), (2, 2, 2))
    S.write_array(p, np.zeros((4, 4, 4), np.uint8))
    assert (p / "c" / "1" / "1" / "1").exists()


def test_reads_v2_style_keys(tmp_path):
    p = tmp_path / "v2.zarr"
    S.create_array(p, "int16", (4, 4), (2, 2))
    S.write_array(p, np.arange(16, dtype=np.int16).reshape(4, 4))
    meta = json.load(open(p / "zarr.json"))
    # rename the chunks to the v2 key encoding with "." and rewrite the metadata
    for i in range(2):
        for j in range(2):
            os.rename(p / "c" / str(i) / str(j), p / f"{i}.{j}")
    meta["chunk_key_encoding"] = {"name": "v2", "configuration": {"separator": "."}}
    json.dump(meta, open(p / "zarr.json", "w"))
    np.testing.assert_array_equal(S.read_array(p), np.arange(16, dtype=np.int16).reshape(4, 4))


def test_big_endian_bytes_codec(tmp_path):
    p = tmp_path / "be.zarr"
    chain = json.dumps([{"name": "bytes", "configuration": {"endian": "big"}}])
    S.create_array(p, "int32", (5,), (5,), chain)
    d = np.array([1, -2, 3, 70000, -5], np.int32)
    S.write_array(p, d)
    assert (p / "c" / "0").read_bytes() == d.astype(">i4").tobytes()
    np.testing.assert_array_equal(S.read_array(p), d)


def test_synthetic_store_matches_oracle(tmp_path):
    shape, chunk = (12, 20, 24), (5, 8, 16)
    p = tmp_path / "syn.zarr"
    S.create_array(p, "float32", shape, chunk)
    S.write_synth(p, S.SYNTH_STEP_NOISE_F32)
    np.testing.assert_array_equal(S.read_array(p), O.synth_step_noise_f32(shape))
    q = tmp_path / "syn16.zarr"
    S.create_array(q, "uint16", shape, chunk)
    S.write_synth(q, S.SYNTH_U16)
    np.testing.assert_array_equal(S.read_array(q), O.synth_u16(shape))


def test_errors_are_filter_errors(tmp_path):
    with pytest.raises(_abi.FilterError, match="zarr.json"):
        S.open_array(tmp_path / "nope")
    p = tmp_path / "bad.zarr"
    p.mkdir()
    (p / "zarr.json").write_text('{"zarr_format": 3, "node_type": "array", "shape": [2],'
                                 '"data_type": "complex64", "chunk_grid": {"name": "regular",'
                                 '"configuration": {"chunk_shape": [2]}}, "chunk_key_encoding":'
                                 '{"name": "default"}, "fill_value": 0, "codecs": '
                                 '[{"name": "bytes"}]}')
    with pytest.raises(_abi.UnsupportedDataType):
        S.open_array(p)
    with pytest.raises(_abi.FilterError):
        S.write_array(S.create_array(tmp_path / "w.zarr", "uint8", (4,), (2,)).path,
                      np.zeros(3, np.uint8), start=(1,))  # not chunk aligned
