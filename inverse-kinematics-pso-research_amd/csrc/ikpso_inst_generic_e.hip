// ikpso_inst_generic_e.hip -- kernel instantiations for generic trees of 13, 14 joints.
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_OTHERS
template struct ModeOps<TopoGeneric<13>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<13>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<14>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<14>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
