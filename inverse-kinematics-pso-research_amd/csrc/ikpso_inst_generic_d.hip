// ikpso_inst_generic_d.hip -- kernel instantiations for generic trees of 11, 12 joints.
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_OTHERS
template struct ModeOps<TopoGeneric<11>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<11>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<12>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<12>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
