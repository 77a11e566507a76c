// g4_limits.hpp — host-side launch limits of the 4-D t-march (guided4d.hip), kept free of HIP
// headers so the host unit test (tests/test_g4_limits.py) compiles them with g++ alone.
#pragma once

#include <stdint.h>

#ifndef G4_TM_MZ
#define G4_TM_MZ 12  // t-march tile depth (tools/timetshare.hip A/B: 12 beats 8 by 4 %)
#endif

namespace zt {

constexpr int kG4TmarchTileZ = G4_TM_MZ;

// Host check of the t-march's 32-bit offsets. The staged offsets (soff) and the v offsets (voff)
// are built from the GLOBAL (y, x) of an element, relative to a per-step z-plane base, so they
// span up to SZ - 1 (= tile z + 2R - 1) planes of z stride plus a whole plane's (ny - 1) rows of
// y stride plus nx elements, not one tile's; TAB offsets span tile-z planes of ny * nx pairs. Any
// span of 2 GiB or more would wrap the (int) offset, and the buffer access would then read 0
// silently. vs3 = the block's (t, z, y) element strides (x stride 1).
inline bool g4_tmarch_offsets_fit(const int64_t* vs3, int ny, int nx, int radius) {
    const int64_t sz = kG4TmarchTileZ + 2 * radius;
    const int64_t v_span = ((sz - 1) * vs3[1] + (int64_t)(ny - 1) * vs3[2] + nx) * 4;
    const int64_t t_span = ((int64_t)kG4TmarchTileZ * ny * nx) * 8;
    return v_span < ((int64_t)1 << 31) && t_span < ((int64_t)1 << 31);
}

}  // namespace zt
