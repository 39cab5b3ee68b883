// Hand-off stencil kernels of fused depth 16, tail offset 6 (life_stencil.h).
#include "life_stencil.h"

namespace gol {
GOL_INSTANTIATE_HAND(16, 6)
}  // namespace gol
