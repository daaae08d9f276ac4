// ikpso_inst_generic_d.hip -- kernel instantiations (generated layout: one unit per
// heavy (topology, mode[, family]) so the build parallelises).
#include "ikpso_topo_impl.h"

namespace ikpso {
#ifndef IKPSO_EXPERIMENT_REF7_ONLY
template struct ModeOps<TopoGeneric<12>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoGeneric<12>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
