// ikpso_inst_generic_g.hip -- kernel instantiations for generic trees of 17, 18 joints.
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_OTHERS
template struct ModeOps<TopoGeneric<17>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<17>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<18>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<18>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
