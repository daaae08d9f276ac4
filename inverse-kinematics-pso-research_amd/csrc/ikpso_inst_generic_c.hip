// ikpso_inst_generic_c.hip -- kernel instantiations for generic trees of 9, 10 joints.
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_OTHERS
template struct ModeOps<TopoGeneric<9>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<9>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<10>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<10>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
