// ikpso_inst_ref7_ref.hip -- kernel instantiations (generated layout: one unit per
// heavy (topology, mode[, family]) so the build parallelises).
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_REF7
template struct ModeOps<TopoRef7, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
