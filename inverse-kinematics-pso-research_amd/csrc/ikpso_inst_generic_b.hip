// ikpso_inst_generic_b.hip -- kernel instantiations for generic trees of 6, 7, 8 joints.
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_OTHERS
template struct ModeOps<TopoGeneric<6>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<6>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<7>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<7>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<8>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<8>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
