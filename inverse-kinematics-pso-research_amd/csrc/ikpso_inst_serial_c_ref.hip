// ikpso_inst_serial_c_ref.hip -- kernel instantiations for serial chains of 12, 13, 14 joints with a tip
// effector (DH arms built by ikpso.dh).
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_DH
template struct ModeOps<TopoSerialTip<12>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoSerialTip<13>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoSerialTip<14>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
