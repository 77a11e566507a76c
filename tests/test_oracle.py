"""CPU: the oracle (oracle/zt_oracle.c) against the reference's own known-answer tests and the
committed golden fixtures. These pin the restatement before it is trusted as the checker."""
import numpy as np
import pytest

from oracle import oracle as O

# guided_filter.rs:364-369
KAT_GUIDED = np.array([[1.659829, 2.1910257, 2.5641026, 3.0],
                       [2.1910257, 2.614423, 3.0, 3.4358974],
                       [2.5641026, 3.0, 3.385577, 3.8089743],
                       [3.0, 3.4358974, 3.8089743, 4.340171]], dtype=np.float32)


def kat_input():
    # guided_filter.rs:342-347: value = row + col, 4x4 f32
    return np.array([[i + j for j in range(4)] for i in range(4)], dtype=np.float32)


def test_guided_filter_kat_chunked_bit_exact():
    # GuidedFilter::new(1.0, 2, None).apply on 2x2 chunks (guided_filter.rs:356-371)
    out = O.guided_filter_apply(kat_input(), (2, 2), 1.0, 2)
    assert np.array_equal(out, KAT_GUIDED)


def test_guided_filter_kat_faithful_mode_same_result():
    out = O.guided_filter_apply(kat_input(), (2, 2), 1.0, 2, faithful=True)
    assert np.array_equal(out, KAT_GUIDED)


def test_guided_filter_box_variance_form_does_not_match():
    # the textbook (windowed variance) form misses the golden values; the
    # pointwise-variance restatement is the one the reference computes.
    v = kat_input().astype(np.float64)
    n = 4
    r = 2

    def box(a):
        o = np.empty_like(a)
        for i in range(n):
            for j in range(n):
                sl = a[max(i - r, 0):min(i + r, n - 1) + 1, max(j - r, 0):min(j + r, n - 1) + 1]
                o[i, j] = sl.mean()
        return o
    u = box(v)
    var = box((v - u) ** 2)
    a = var / (var + 1.0)
    b = (1 - a) * u
    out = v * box(a) + box(b)
    assert np.abs(out - KAT_GUIDED).max() > 0.1


def test_summed_area_table_kat():
    # summed_area_table.rs:276-313 (u8 6x6 -> integral image)
    a = np.array([[31, 2, 4, 33, 5, 36], [12, 26, 9, 10, 29, 25], [13, 17, 21, 22, 20, 18],
                  [24, 23, 15, 16, 14, 19], [30, 8, 28, 27, 11, 7], [1, 35, 34, 3, 32, 6]],
                 dtype=np.float32)
    ref = np.array([[31, 33, 37, 70, 75, 111], [43, 71, 84, 127, 161, 222],
                    [56, 101, 135, 200, 254, 333], [80, 148, 197, 278, 346, 444],
                    [110, 186, 263, 371, 450, 555], [111, 222, 333, 444, 555, 666]])
    assert np.array_equal(O.summed_area_table(a), ref)


def test_chunking_matches_whole_block_halo_is_sufficient():
    # a 2r halo makes the chunked result equal to the whole-volume result.
    v = O.synth_step_noise_f32((12, 12, 12))
    whole = O.guided_filter_apply_ndarray(v, 2500.0, 2)
    chunked = O.guided_filter_apply(v, (4, 4, 4), 2500.0, 2, nthreads=4)
    assert np.abs(whole - chunked).max() <= 1e-5 * np.abs(whole).max()


@pytest.mark.parametrize("value,bits", [
    (1.0, 0x3C00), (65504.0, 0x7BFF), (65520.0, 0x7C00), (-2.0, 0xC000),
    (5.960464477539063e-08, 0x0001), (1e-9, 0x0000), (float("inf"), 0x7C00),
    (1.0009765625, 0x3C01), (1.00048828125, 0x3C00),  # tie -> even
])
def test_f32_to_f16_half_crate(value, bits):
    assert int(O.cast_from_f32(np.array([value], np.float32), "float16")[0]) == bits


@pytest.mark.parametrize("value,bits", [
    (1.0, 0x3F80), (1.00390625, 0x3F80), (1.01171875, 0x3F82), (-3.5, 0xC060),
    (3.4028234663852886e38, 0x7F80),
])
def test_f32_to_bf16_half_crate(value, bits):
    assert int(O.cast_from_f32(np.array([value], np.float32), "bfloat16")[0]) == bits


def test_nan_casts():
    nan = np.array([np.nan], np.float32)
    assert int(O.cast_from_f32(nan, "float16")[0]) & 0x7E00 == 0x7E00
    assert int(O.cast_from_f32(nan, "bfloat16")[0]) & 0x7FC0 == 0x7FC0
    for d in ("uint8", "int8", "int32", "uint64", "int64"):
        assert int(O.cast_from_f32(nan, d)[0]) == 0


@pytest.mark.parametrize("dtype,vals,expect", [
    ("uint8", [300.7, -5.5, 2.9, 255.99], [255, 0, 2, 255]),
    ("int8", [-2.9, 127.5, -200.0], [-2, 127, -128]),
    ("int32", [1e10, -1e10, -7.9], [2147483647, -2147483648, -7]),
    ("uint16", [65535.9, 65536.0, 0.99], [65535, 65535, 0]),
    ("uint64", [1.8446744073709552e19, 5.5], [18446744073709551615, 5]),
])
def test_rust_as_saturating_casts(dtype, vals, expect):
    out = O.cast_from_f32(np.array(vals, np.float32), dtype)
    assert [int(x) for x in out] == expect


def test_downsample_integer_mean_truncates():
    v = np.array([[1, 2], [2, 2]], dtype=np.uint16)  # mean 1.75 -> `as u16` = 1
    assert O.downsample(v, "uint16", (2, 2), "uint16")[0, 0] == 1
    assert O.downsample(v, "uint16", (2, 2), "float32")[0, 0] == np.float32(1.75)


def test_downsample_drops_partial_windows():
    v = np.arange(5 * 3, dtype=np.float32).reshape(5, 3)
    out = O.downsample(v, "float32", (2, 2), "float32")
    assert out.shape == (2, 1)
    assert out[1, 0] == np.float32((6 + 7 + 9 + 10) / 4)


def test_downsample_short_axis_window_is_extent():
    # downsample.rs:83-85: window = min(stride, extent)
    v = np.arange(3 * 4, dtype=np.float32).reshape(3, 4)
    out = O.downsample(v, "float32", (4, 2), "float32")
    assert out.shape == (1, 2)
    assert out[0, 0] == np.float32(np.mean([0, 1, 4, 5, 8, 9]))


def test_downsample_mode_tie_smallest():
    v = np.array([[3, 1], [1, 3]], dtype=np.uint8)
    assert O.downsample(v, "uint8", (2, 2), "uint8", discrete=True)[0, 0] == 1


@pytest.mark.parametrize("dtype", ["int64", "uint64"])
def test_downsample_mode_64bit_keys_exact(dtype):
    """downsample.rs:113-117 counts exact `TIn` keys (HashMap<TIn, usize>): two 64-bit values
    that are equal as f64 must stay distinct keys, and the winner comes back unrounded."""
    a = 2 ** 62 + 1            # a, b: one f64 (2^62), distinct integers
    b = 2 ** 62 + 3
    c = 2 ** 62 + 2 ** 11      # the next f64 above 2^62
    assert float(a) == float(b)
    # three b, one a: b wins (as f64 keys all four would tie and come back as 2^62)
    v = np.array([[a, b], [b, b]], dtype=dtype)
    out = O.downsample(v, dtype, (2, 2), dtype, discrete=True)
    assert int(out[0, 0]) == b
    # two a, two b: a tie between distinct keys goes to the smaller value
    v = np.array([[b, a], [a, b]], dtype=dtype)
    assert int(O.downsample(v, dtype, (2, 2), dtype, discrete=True)[0, 0]) == a
    # integer -> f32 rounds once (`as`): c is exactly representable
    v = np.array([[c, c], [a, b]], dtype=dtype)
    assert O.downsample(v, dtype, (2, 2), "float32", discrete=True)[0, 0] == np.float32(c)
    # signed order for the tie: -1 < 1 (as uint64 bits -1 would be the larger)
    if dtype == "int64":
        v = np.array([[1, -1], [-1, 1]], dtype=dtype)
        assert int(O.downsample(v, dtype, (2, 2), dtype, discrete=True)[0, 0]) == -1


def test_synthetic_generator_definition():
    v = O.synth_step_noise_f32((2, 3, 8))
    h = O.lib().oracle_splitmix64(O.SEED ^ 5)
    u = np.float32(h >> 40) * np.float32(2.0 ** -24)
    assert v.reshape(-1)[5] == np.float32(np.float32(100.0) * u) + np.float32(500.0)
    assert (v[..., :4] < 100).all() and (v[..., 4:] >= 500).all()


def test_golden_fixtures_reproduce(golden_cases, golden_dir):
    import os
    for c in golden_cases["guided_filter"]:
        vin = np.load(os.path.join(golden_dir, c["name"] + "_in.npy"))
        exp = np.load(os.path.join(golden_dir, c["name"] + "_out_f32.npy"))
        v32 = vin if c["dtype_in"] == "float32" else O.cast_to_f32(vin, c["dtype_in"])
        out = O.guided_filter_apply(v32, c["chunk_shape"], c["epsilon"], c["radius"], nthreads=4)
        assert np.array_equal(out, exp), c["name"]
    for c in golden_cases["downsample"]:
        vin = np.load(os.path.join(golden_dir, c["name"] + "_in.npy"))
        exp = np.load(os.path.join(golden_dir, c["name"] + "_out.npy"))
        out = O.downsample(vin, c["dtype_in"], c["stride"], c["dtype_out"], c["discrete"])
        assert np.array_equal(out, exp), c["name"]
