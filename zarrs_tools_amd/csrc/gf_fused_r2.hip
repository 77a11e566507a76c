// gf_fused_r2.hip — fused guided-filter instantiations for radius 2.
#include "gf_fused.hpp"

namespace zt {
ZT_FUSED_PAIRS(2, 32, 1024)
}  // namespace zt
