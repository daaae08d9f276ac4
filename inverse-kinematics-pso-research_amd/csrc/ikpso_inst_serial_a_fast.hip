// ikpso_inst_serial_a_fast.hip -- kernel instantiations for serial chains of 6, 7, 8 joints with a tip
// effector (DH arms built by ikpso.dh).
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_DH
template struct ModeOps<TopoSerialTip<6>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoSerialTip<7>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoSerialTip<8>, IKPSO_ARITH_FAST>;
#endif
}  // namespace ikpso
