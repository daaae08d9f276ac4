// ikpso_inst_serial20_coop_ref.hip -- kernel instantiations (generated layout: one unit per
// heavy (topology, mode[, family]) so the build parallelises).
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_SERIAL20
template hipError_t ModeOps<TopoSerialTip<20>, IKPSO_ARITH_REFERENCE>::coop(const ChainHost&, const SwarmIO&, hipStream_t);
#endif
}  // namespace ikpso
