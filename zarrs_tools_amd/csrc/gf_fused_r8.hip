// gf_fused_r8.hip — fused guided-filter instantiations for radius 8.
#include "gf_fused.hpp"

namespace zt {
ZT_FUSED_PAIRS(8, 16, 1024)
}  // namespace zt
