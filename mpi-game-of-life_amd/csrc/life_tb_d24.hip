// Stencil kernels of fused depth 24 (dev build only: make dev); see life_stencil.h.
#include "life_stencil.h"

#if GOL_DEV_KERNELS
namespace gol {
GOL_INSTANTIATE_DEPTH(24)
}  // namespace gol
#endif
