// gf_fused_r3.hip — fused guided-filter instantiations for radius 3.
#include "gf_fused.hpp"

namespace zt {
ZT_FUSED_PAIRS(3, 32, 1024)
}  // namespace zt
