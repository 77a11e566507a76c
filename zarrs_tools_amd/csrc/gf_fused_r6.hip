// gf_fused_r6.hip — fused guided-filter instantiations for radius 6.
#include "gf_fused.hpp"

namespace zt {
ZT_FUSED_PAIRS(6, 16, 1024)
}  // namespace zt
