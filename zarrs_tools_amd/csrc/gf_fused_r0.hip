// gf_fused_r0.hip — fused guided-filter instantiations for radius 0.
#include "gf_fused.hpp"

namespace zt {
ZT_FUSED_PAIRS(0, 32, 1024)
}  // namespace zt
