// gf_fused_r1.hip — fused guided-filter instantiations for radius 1.
#include "gf_fused.hpp"

namespace zt {
ZT_FUSED_PAIRS(1, 32, 1024)
}  // namespace zt
