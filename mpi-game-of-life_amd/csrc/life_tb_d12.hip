// Stencil kernels of fused depth 12: classic row blocks and the dispatch; the
// hand-off kernels (tail offsets 0 and 2) compile in life_tb_d12h0.hip and
// life_tb_d12h2.hip.  See life_stencil.h.
#include "life_stencil.h"

namespace gol {
GOL_EXTERN_HAND(12, 0)
GOL_EXTERN_HAND(12, 2)
GOL_INSTANTIATE_DEPTH(12)
}  // namespace gol
