// ikpso_inst_generic_f.hip -- kernel instantiations for generic trees of 15, 16 joints.
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_OTHERS
template struct ModeOps<TopoGeneric<15>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<15>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoGeneric<16>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<16>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
