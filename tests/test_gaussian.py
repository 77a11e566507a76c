"""Gaussian (gaussian.rs, kernel.rs) on the CPU: the oracle against the reference's known-answer
test, the tap generator of the C ABI against the oracle's, and the halo property that lets the
GPU run one pass over a whole array instead of a loop over chunks."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

# gaussian.rs:277-321: 4x4 f32 (i + j), chunks 2x2, sigma 1, kernel half size 3
KAT_IN = np.array([[i + j for j in range(4)] for i in range(4)], dtype=np.float32)
KAT_OUT = np.array([[0.7262998, 1.4210157, 2.3036606, 2.9983768],
                    [1.4210159, 2.1157317, 2.9983768, 3.6930926],
                    [2.3036606, 2.9983766, 3.8810213, 4.575738],
                    [2.9983768, 3.6930926, 4.5757375, 5.2704535]], dtype=np.float32)


def test_oracle_reproduces_reference_kat_bit_exactly():
    out = O.gaussian_apply(KAT_IN, (2, 2), [1.0, 1.0], [3, 3])
    assert np.array_equal(out, KAT_OUT)


def test_kernel_taps_follow_the_reference_formula():
    for sigma, half in [(1.0, 3), (0.5, 2), (2.5, 8), (0.0, 3), (1.7, 0)]:
        taps = O.gaussian_kernel(sigma, half)
        if sigma == 0.0:
            assert taps.tolist() == [1.0]
            continue
        assert len(taps) == 2 * half + 1
        assert np.array_equal(taps, taps[::-1])
        t = np.float32(sigma) * np.float32(sigma)
        scale = np.float32(1.0) / np.sqrt(np.float32(2.0) * np.float32(np.pi) * t)
        n = np.arange(half + 1, dtype=np.float32)
        ref = scale * np.exp(-(n * n) / (np.float32(2.0) * t))
        # numpy's exp may differ from libm expf by an ulp: the formula, not the bits, here
        np.testing.assert_allclose(taps[half:], ref, rtol=3e-7)


def test_library_taps_equal_oracle_taps():
    import zarrs_tools_amd as zt  # host-only entry point: no GPU needed
    lib = zt._abi.lib()
    for sigma, half in [(1.0, 3), (0.5, 2), (2.5, 8), (0.0, 3), (3.3, 10), (12.0, 36)]:
        n = ctypes.c_int64()
        assert lib.zt_gaussian_kernel(sigma, half, None, ctypes.byref(n)) == 0
        taps = (ctypes.c_float * n.value)()
        assert lib.zt_gaussian_kernel(sigma, half, taps, ctypes.byref(n)) == 0
        assert np.array_equal(np.array(taps[:], np.float32), O.gaussian_kernel(sigma, half))


@pytest.mark.parametrize("shape,chunk,sigma,half", [
    ((23,), (5,), [1.3], [4]),
    ((9, 17), (4, 5), [1.0, 0.7], [3, 2]),
    ((7, 10, 13), (3, 4, 5), [1.2, 0.0, 2.0], [4, 3, 6]),
    ((4, 5, 6, 7), (2, 3, 4, 3), [0.8, 1.0, 1.5, 0.5], [2, 3, 5, 1]),
])
def test_chunked_equals_whole_block(shape, chunk, sigma, half):
    # a kernel_half_size halo clamped to the array makes every chunk's windows clamp exactly where
    # the whole array's do, so the chunk loop equals one pass (what zt_gaussian_apply_array runs)
    rng = np.random.default_rng(len(shape))
    v = (rng.random(shape, dtype=np.float32) * 100).astype(np.float32)
    assert np.array_equal(O.gaussian_apply(v, chunk, sigma, half),
                          O.gaussian_apply_ndarray(v, sigma, half))
