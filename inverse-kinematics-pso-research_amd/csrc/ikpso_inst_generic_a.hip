// ikpso_inst_generic_a.hip -- kernel instantiations for generic trees of 1, 2, 3, 4, 5 joints.
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_OTHERS
template struct ModeOps<TopoGeneric<1>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<1>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<2>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<2>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<3>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<3>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<4>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<4>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<5>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<5>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
