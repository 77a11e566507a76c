"""CPU: the 4-D t-march's 32-bit offset check (g4_tmarch_offsets_fit, zarrs_tools_amd/csrc/
g4_limits.hpp) at the boundary shapes. The t-march (guided4d.hip) forms its staged
and v offsets from the GLOBAL (y, x) of an element relative to a z-plane base, and its TAB
offsets over whole planes; a block whose offsets reach 2 GiB must take the K1 + g4_tab path, or
the buffer loads past the wrap read 0 silently. The predicate is compiled here with g++ (the
header has no HIP dependency) and compared with the largest offsets the kernel's index formulas
produce, for contiguous blocks at the bound and for strided views (large y / z strides)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zarrs_tools_amd", "csrc")

DRIVER = r"""
#include <cstdio>
#include "g4_limits.hpp"
int main() {
    std::printf("%d\n", zt::kG4TmarchTileZ);
    long long vt, vz, vy; int ny, nx, r;
    while (std::scanf("%lld %lld %lld %d %d %d", &vt, &vz, &vy, &ny, &nx, &r) == 6) {
        const int64_t vs3[3] = {vt, vz, vy};
        std::printf("%d\n", zt::g4_tmarch_offsets_fit(vs3, ny, nx, r) ? 1 : 0);
    }
    return 0;
}
"""


@pytest.fixture(scope="module")
def predicate(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("g4lim")
    src, exe = d / "drv.cpp", d / "drv"
    src.write_text(DRIVER)
    subprocess.run([gxx, "-O1", "-std=c++17", "-I", CSRC, str(src), "-o", str(exe)], check=True)

    def run(cases):
        inp = "".join(f"{vt} {vz} {vy} {ny} {nx} {r}\n" for vt, vz, vy, ny, nx, r in cases)
        out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True,
                             check=True).stdout.split()
        return int(out[0]), [o == "1" for o in out[1:]]
    return run


def kernel_offsets_fit(vz, vy, ny, nx, r, tile_z):
    """The largest byte offsets g4_tmarch_tab_kernel forms, from its index formulas:
    staged v: ((ez + zsh) * vs.z + gy * vs.y + gx) * 4 with ez + zsh <= tile_z + 2r - 1,
    gy <= ny - 1, gx <= nx - 1 (a 4-byte access); v(tau) at the thread's voxels lies inside that;
    TAB: (((lz + q) * ny + gy) * nx + gx) * 8 with lz + q <= tile_z - 1 (an 8-byte access).
    Every access must end below 2^31 (the int offset must not wrap)."""
    v_end = ((tile_z + 2 * r - 1) * vz + (ny - 1) * vy + (nx - 1)) * 4 + 4
    t_end = (((tile_z - 1) * ny + (ny - 1)) * nx + (nx - 1)) * 8 + 8
    return v_end < 2 ** 31 and t_end < 2 ** 31


def test_tmarch_offsets_fit_boundary_shapes(predicate):
    tile_z, _ = predicate([])
    cases = []
    for r in (1, 2):
        # contiguous blocks: TAB's tile_z planes bind first (ny * nx < 2^28 / tile_z)
        lim = (2 ** 28 - 1) // tile_z
        for plane in (lim - 1, lim, lim + 1, lim + 4096, 33_554_432, 35_800_000, 41_300_000):
            for nx in (4096, 8192, 1024):
                ny = plane // nx
                if ny < 1:
                    continue
                cases.append((40 * ny * nx, ny * nx, nx, ny, nx, r))
        # strided views (in-place sub-arrays of a larger tensor): large y / z strides, small planes
        for vy in (2048, 1 << 20, (1 << 21) + 7, 1 << 22):
            for ny in (64, 256, 511, 512, 1024):
                nx = 256
                vz = vy * (ny + 3)
                cases.append((vz * 24, vz, vy, ny, nx, r))
    _, got = predicate(cases)
    want = [kernel_offsets_fit(vz, vy, ny, nx, r, tile_z) for _, vz, vy, ny, nx, r in cases]
    assert got == want
    assert any(got) and not all(got)  # both sides of the bound are exercised


def test_tmarch_offsets_plane_span_not_tile_span(predicate):
    """ADVICE r5's case: a bound on one tile's span (SZ - 1 planes + one tile of rows) passes a
    block whose real offsets, built from the global y, wrap; the predicate must refuse it."""
    tile_z, _ = predicate([])
    r, nx, vy = 2, 256, 2048  # a strided view: rows 2048 elements apart
    sz = tile_z + 2 * r
    # the largest plane stride a one-tile bound accepts, and a plane whose rows fill it
    vz = ((2 ** 31) // 4 - (16 + 2 * r) * vy - 64) // (sz - 1)
    ny = (vz - nx) // vy
    tile_span = ((sz - 1) * vz + (16 + 2 * r - 1) * vy + 16 + 2 * r) * 4
    assert tile_span < 2 ** 31
    assert not kernel_offsets_fit(vz, vy, ny, nx, r, tile_z)
    _, got = predicate([(vz * 24, vz, vy, ny, nx, r)])
    assert got == [False]
