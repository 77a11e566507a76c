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


# ---- byte layouts pinned against the Zarr V3 specification and independent decoders ----------
# (the reference ships no store fixtures; these check the chunks this store writes with decoders
# that share no code with it: Python's gzip / zlib, a table-free crc32c, libzstd through ctypes)

def _crc32c(data: bytes) -> int:
    """CRC-32C (Castagnoli, reflected polynomial 0x82F63B78), bit by bit."""
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def test_crc32c_reference_value():
    assert _crc32c(b"123456789") == 0xE3069283  # the CRC-32C check value


def _chunk(data, idx, chunk):
    sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(idx, chunk))
    blk = data[sl]
    out = np.zeros(chunk, data.dtype)  # edge chunks are padded with the fill value (0)
    out[tuple(slice(0, n) for n in blk.shape)] = blk
    return out


def test_gzip_chunks_decode_with_python_gzip(tmp_path):
    import gzip
    shape, chunk = (10, 12), (8, 8)
    p = tmp_path / "g.zarr"
    S.create_array(p, "int16", shape, chunk, S.codecs_json("gzip", 6))
    data = np.arange(120, dtype=np.int16).reshape(shape) * 7 - 300
    S.write_array(p, data)
    for i in range(2):
        for j in range(2):
            raw = gzip.decompress((p / "c" / str(i) / str(j)).read_bytes())
            assert raw == _chunk(data, (i, j), chunk).astype("<i2").tobytes()


def test_zstd_chunks_decode_with_libzstd(tmp_path):
    import ctypes
    import ctypes.util
    if not S.codec_available("zstd"):
        pytest.skip("libzstd.so.1 not present")
    z = ctypes.CDLL(ctypes.util.find_library("zstd") or "libzstd.so.1")
    z.ZSTD_decompress.restype = ctypes.c_size_t
    z.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                  ctypes.c_size_t]
    z.ZSTD_isError.argtypes = [ctypes.c_size_t]
    shape, chunk = (9, 9), (9, 9)
    p = tmp_path / "z.zarr"
    S.create_array(p, "float32", shape, chunk, S.codecs_json("zstd", 3))
    data = np.linspace(-4, 4, 81, dtype=np.float32).reshape(shape)
    S.write_array(p, data)
    comp = (p / "c" / "0" / "0").read_bytes()
    assert comp[:4] == b"\x28\xb5\x2f\xfd"  # zstd frame magic
    out = ctypes.create_string_buffer(data.nbytes)
    n = z.ZSTD_decompress(out, data.nbytes, comp, len(comp))
    assert not z.ZSTD_isError(n) and n == data.nbytes
    assert out.raw == data.astype("<f4").tobytes()


def test_sharding_layout_per_spec(tmp_path):
    """sharding_indexed, index at the end: n inner chunks x (offset u64 LE, nbytes u64 LE), the
    index bytes followed by their crc32c (u32 LE); empty inner chunks are (2^64-1, 2^64-1)."""
    import struct
    p = tmp_path / "s.zarr"
    inner = (4, 4)
    S.create_array(p, "uint16", (8, 8), (8, 8), S.codecs_json(shard_inner=inner))
    data = np.arange(64, dtype=np.uint16).reshape(8, 8)
    data[4:, 4:] = 0  # may be stored as an empty inner chunk (all fill value)
    S.write_array(p, data)
    raw = (p / "c" / "0" / "0").read_bytes()
    n = 4
    index = raw[-(16 * n + 4):-4]
    assert struct.unpack("<I", raw[-4:])[0] == _crc32c(index)
    for k in range(n):
        off, nb = struct.unpack("<QQ", index[16 * k:16 * k + 16])
        i, j = divmod(k, 2)  # C order over the inner chunk grid
        want = _chunk(data, (i, j), inner)
        if off == 2 ** 64 - 1:
            assert nb == 2 ** 64 - 1 and not want.any()
            continue
        assert raw[off:off + nb] == want.astype("<u2").tobytes()


def test_crc32c_codec_appends_checksum(tmp_path):
    import struct
    p = tmp_path / "c.zarr"
    chain = json.dumps([{"name": "bytes", "configuration": {"endian": "little"}},
                        {"name": "crc32c"}])
    S.create_array(p, "uint8", (16,), (16,), chain)
    data = np.arange(16, dtype=np.uint8) * 3
    S.write_array(p, data)
    raw = (p / "c" / "0").read_bytes()
    assert raw[:-4] == data.tobytes()
    assert struct.unpack("<I", raw[-4:])[0] == _crc32c(data.tobytes())
