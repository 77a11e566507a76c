"""GPU parity of the single-barrier fused kernel (gf_v9.hpp) against the oracle.

gf3d_v9_kernel is opt-in (zt_set_fused_variant(1); the default kernel is faster)
and takes radius 1..4 launches whose x geometry is quad aligned (x extent, x origin of the output
box and row pitches multiples of 4). The module selects it for its own tests and restores the
default afterwards. Cases: partial tiles in x and y, tiles touching every face of the domain,
windows clamped on both sides, per-chunk launches (the x origin of a chunk is a multiple of 4),
and the direct u16 / u8 element-type pairs. Tolerance as DESIGN.md §4.
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.gpu_util import FLOAT_TOL, rel_err
from tests.test_guided_filter_gpu import check_against, gpu_apply, gpu_apply_chunked

pytestmark = pytest.mark.gpu

import zarrs_tools_amd as zt  # noqa: E402,F401  (no skip: the HIP library must load)
from zarrs_tools_amd import _abi  # noqa: E402


@pytest.fixture(autouse=True, scope="module")
def _select_v9():
    prev = _abi.lib().zt_set_fused_variant(1)
    yield
    _abi.lib().zt_set_fused_variant(prev)


@pytest.mark.parametrize("r", [1, 2, 3, 4])
@pytest.mark.parametrize("eps", [0.5, 2500.0])
def test_v9_radii(r, eps):
    rng = np.random.default_rng(100 + r)
    shape = (int(rng.integers(2 * r + 3, 24)), int(rng.integers(5, 75)),
             4 * int(rng.integers(2, 40)))
    chunk = (int(rng.integers(3, 12)), int(rng.integers(4, 40)), 4 * int(rng.integers(1, 12)))
    v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
    ref = O.guided_filter_apply(v, chunk, eps, r, nthreads=8)
    out = gpu_apply(v, "float32", "float32", chunk, eps, r)
    assert rel_err(out, ref) <= FLOAT_TOL, (shape, chunk)


@pytest.mark.parametrize("shape", [(1, 1, 4), (3, 2, 8), (5, 33, 64), (9, 31, 68),
                                   (12, 65, 132), (20, 40, 196)])
def test_v9_shapes_r4(shape):
    v = O.synth_step_noise_f32(shape)
    chunk = (4, 16, 32)
    ref = O.guided_filter_apply(v, chunk, 2500.0, 4, nthreads=8)
    out = gpu_apply(v, "float32", "float32", chunk, 2500.0, 4)
    assert rel_err(out, ref) <= FLOAT_TOL


@pytest.mark.parametrize("r", [2, 4])
def test_v9_per_chunk(r):
    v = O.synth_step_noise_f32((14, 45, 100))
    chunk = (5, 16, 20)
    ref = O.guided_filter_apply(v, chunk, 50.0, r, nthreads=8)
    out = gpu_apply_chunked(v, "float32", "float32", chunk, 50.0, r)
    assert rel_err(out, ref) <= FLOAT_TOL


@pytest.mark.parametrize("din,dout", [("uint16", "float32"), ("uint8", "float32"),
                                      ("float32", "uint16"), ("uint16", "uint16"),
                                      ("uint8", "uint8")])
def test_v9_element_types(din, dout):
    rng = np.random.default_rng(5)
    shape = (10, 37, 136)
    scale = 250.0 if "uint8" in (din, dout) else 4000.0
    v = O.cast_from_f32((rng.random(shape, dtype=np.float32) * scale).astype(np.float32), din)
    ref = O.guided_filter_apply(O.cast_to_f32(v, din), (8, 16, 64), 100.0, 3, nthreads=8)
    out = gpu_apply(v, din, dout, (8, 16, 64), 100.0, 3)
    check_against(out, ref, dout)


def test_v9_large_values_and_constant_regions():
    # constant blocks give s = 0 -> a = 0 (0/eps); large values stress the exact f64 stage 1
    v = np.zeros((12, 40, 128), np.float32)
    v[:, :, 64:] = 3.0e6
    v[4:8, 10:30, 20:100] += np.float32(1.0e-3) * np.arange(80, dtype=np.float32)
    ref = O.guided_filter_apply(v, (6, 20, 64), 0.5, 4, nthreads=8)
    out = gpu_apply(v, "float32", "float32", (6, 20, 64), 0.5, 4)
    assert rel_err(out, ref) <= FLOAT_TOL
