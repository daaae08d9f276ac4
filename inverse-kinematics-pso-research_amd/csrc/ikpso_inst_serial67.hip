// ikpso_inst_serial67.hip -- kernel instantiations for 6- and 7-joint serial
// arms with a tip effector (e.g. DH arms built by ikpso.dh).
#include "ikpso_topo_impl.h"

namespace ikpso {
#if IKPSO_WITH_OTHERS
template struct ModeOps<TopoSerialTip<6>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoSerialTip<6>, IKPSO_ARITH_REFERENCE>;
template struct ModeOps<TopoSerialTip<7>, IKPSO_ARITH_FAST>;
template struct ModeOps<TopoSerialTip<7>, IKPSO_ARITH_REFERENCE>;
#endif
}  // namespace ikpso
