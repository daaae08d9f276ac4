// ikpso_inst_dh_b.hip -- kernel instantiations for folded serial chains (TopoDH) of 8-12 free angles.
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_DH
template struct ModeOps<TopoDH<8>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoDH<9>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoDH<10>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoDH<11>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoDH<12>, IKPSO_ARITH_FAST>;
#endif
}  // namespace ikpso
