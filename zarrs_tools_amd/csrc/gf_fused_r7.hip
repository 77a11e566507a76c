// gf_fused_r7.hip — fused guided-filter instantiations for radius 7.
#include "gf_fused.hpp"

namespace zt {
ZT_FUSED_PAIRS(7, 16, 1024)
}  // namespace zt
