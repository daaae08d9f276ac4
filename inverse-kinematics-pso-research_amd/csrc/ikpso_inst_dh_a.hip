// ikpso_inst_dh_a.hip -- kernel instantiations for folded serial chains (TopoDH) of 3-7 free angles.
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_DH
template struct ModeOps<TopoDH<3>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoDH<4>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoDH<5>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoDH<6>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoDH<7>, IKPSO_ARITH_FAST>;
#endif
}  // namespace ikpso
