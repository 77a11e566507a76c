// gf_fused_r5.hip — fused guided-filter instantiations for radius 5.
#include "gf_fused.hpp"

namespace zt {
ZT_FUSED_PAIRS(5, 16, 1024)
}  // namespace zt
