// Stencil kernels of fused depth 16: classic row blocks and the dispatch; the
// hand-off kernels (tail offsets 0, 2, 4, 6) compile in life_tb_d16h<offset>.hip.
// See life_stencil.h.
#include "life_stencil.h"

namespace gol {
GOL_EXTERN_HAND(16, 0)
GOL_EXTERN_HAND(16, 2)
GOL_EXTERN_HAND(16, 4)
GOL_EXTERN_HAND(16, 6)
GOL_INSTANTIATE_DEPTH(16)
}  // namespace gol
