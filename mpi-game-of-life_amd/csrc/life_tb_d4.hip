// Stencil kernels of fused depth 4 (all rule kinds, hand-off and classic row
// blocks); see life_stencil.h.  One translation unit per depth keeps builds parallel.
#include "life_stencil.h"

namespace gol {
GOL_INSTANTIATE_DEPTH(4)
}  // namespace gol
