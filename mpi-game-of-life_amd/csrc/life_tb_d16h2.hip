// Hand-off stencil kernels of fused depth 16, tail offset 2 (life_stencil.h).
#include "life_stencil.h"

namespace gol {
GOL_INSTANTIATE_HAND(16, 2)
}  // namespace gol
