// ikpso_topo_impl.h -- definitions of ModeOps<Topo, MODE>; include from the
// ikpso_inst_*.hip translation units, followed by explicit instantiations.
#pragma once

#include "ikpso_coop.h"
#include "ikpso_resident.h"
#include "ikpso_stream.h"
#include "ikpso_topo_ops.h"

namespace ikpso {

template <class Topo, int MODE>
hipError_t ModeOps<Topo, MODE>::resident(const ChainHost& ch, const SwarmIO& io, int block, hipStream_t s)
{
    return run_resident<Topo, MODE>(ch, io, block, s);
}

template <class Topo, int MODE>
hipError_t ModeOps<Topo, MODE>::stream(const ChainHost& ch, const StreamIO& io, int iterations, hipStream_t s)
{
    return run_stream_terms<Topo, MODE>(ch, io, iterations, s);
}

template <class Topo, int MODE>
hipError_t ModeOps<Topo, MODE>::evaluate(const ChainHost& ch, const EvalIO& io, hipStream_t s)
{
    return run_evaluate<Topo, MODE>(ch, io, s);
}

template <class Topo, int MODE>
hipError_t ModeOps<Topo, MODE>::coop(const ChainHost& ch, const SwarmIO& io, hipStream_t s)
{
    if constexpr (Topo::kGeneric)
        return hipErrorNotSupported;  // generic trees take the streaming kernels
    else
        return run_coop<Topo, MODE>(ch, io, s);
}

}  // namespace ikpso
