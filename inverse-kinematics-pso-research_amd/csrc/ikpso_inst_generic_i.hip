// ikpso_inst_generic_i.hip -- kernel instantiations for generic trees of 20 joints.
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_OTHERS
template struct ModeOps<TopoGeneric<20>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<20>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
