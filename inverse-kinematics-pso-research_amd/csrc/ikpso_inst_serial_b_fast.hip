// ikpso_inst_serial_b_fast.hip -- kernel instantiations for serial chains of 9, 10, 11 joints with a tip
// effector (DH arms built by ikpso.dh).
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_DH
template struct ModeOps<TopoSerialTip<9>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoSerialTip<10>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoSerialTip<11>, IKPSO_ARITH_FAST>;
#endif
}  // namespace ikpso
