// Hand-off stencil kernels of fused depth 12, tail offset 2 (life_stencil.h).
#include "life_stencil.h"

namespace gol {
GOL_INSTANTIATE_HAND(12, 2)
}  // namespace gol
