// gf_fused_r4.hip — fused guided-filter instantiations for radius 4.
#include "gf_fused.hpp"

namespace zt {
ZT_FUSED_PAIRS(4, 32, 1024)
}  // namespace zt
