// ikpso_topo_ops.h -- per-topology launch entry points.  The kernel templates
// (ikpso_resident.h, ikpso_stream.h) are instantiated per (topology, mode) in
// their own translation units (ikpso_inst_*.hip) so the build parallelises;
// the dispatcher (ikpso_kernels.hip) sees only these declarations.
#pragma once

#include <hip/hip_runtime.h>

#include "ikpso_kernels.h"

namespace ikpso {

template <class Topo, int MODE>
struct ModeOps {
    static hipError_t resident(const ChainHost& ch, const SwarmIO& io, int block, hipStream_t stream);
    static hipError_t stream(const ChainHost& ch, const StreamIO& io, int iterations, hipStream_t stream);
    static hipError_t evaluate(const ChainHost& ch, const EvalIO& io, hipStream_t stream);
    static hipError_t coop(const ChainHost& ch, const SwarmIO& io, hipStream_t stream);
};

// The folded chain (TopoDH) has FAST kernels only: REFERENCE runs of such a
// chain use its Euler form.
template <class Topo>
struct TopoOps {
    static constexpr bool kRef = !Topo::kDH;
    using Ref = ModeOps<Topo, IKPSO_ARITH_REFERENCE>;
    using Fast = ModeOps<Topo, IKPSO_ARITH_FAST>;
    static hipError_t resident(const ChainHost& ch, int mode, const SwarmIO& io, int block, hipStream_t s)
    {
        if (mode == IKPSO_ARITH_REFERENCE) {
            if constexpr (kRef) return Ref::resident(ch, io, block, s);
            return hipErrorNotSupported;
        }
        return Fast::resident(ch, io, block, s);
    }
    static hipError_t stream(const ChainHost& ch, int mode, const StreamIO& io, int iterations, hipStream_t s)
    {
        if (mode == IKPSO_ARITH_REFERENCE) {
            if constexpr (kRef) return Ref::stream(ch, io, iterations, s);
            return hipErrorNotSupported;
        }
        return Fast::stream(ch, io, iterations, s);
    }
    static hipError_t evaluate(const ChainHost& ch, int mode, const EvalIO& io, hipStream_t s)
    {
        if (mode == IKPSO_ARITH_REFERENCE) {
            if constexpr (kRef) return Ref::evaluate(ch, io, s);
            return hipErrorNotSupported;
        }
        return Fast::evaluate(ch, io, s);
    }
    static hipError_t coop(const ChainHost& ch, int mode, const SwarmIO& io, hipStream_t s)
    {
        if (mode == IKPSO_ARITH_REFERENCE) {
            if constexpr (kRef) return Ref::coop(ch, io, s);
            return hipErrorNotSupported;
        }
        return Fast::coop(ch, io, s);
    }
};

}  // namespace ikpso
