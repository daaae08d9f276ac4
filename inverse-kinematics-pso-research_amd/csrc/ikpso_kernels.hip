// ikpso_kernels.hip -- host-side dispatch of the gfx950 kernels of the PSO
// inverse-kinematics hot path, and the generator-seeding kernel.
//
// Replaces the reference's per-iteration launch chain (src/kernel.cu:279-327:
// initParticlesKernel, initLocalBests, thrust::min_element, a blocking D2H
// copy and updateGlobalBestCoordsKernel per iteration) with ONE launch per
// batch of swarms (k_swarm_resident, ikpso_resident.h) or, for swarms larger
// than a workgroup, one launch per iteration (ikpso_stream.h).  Each compiled
// topology's kernels live in their own translation unit (ikpso_inst_*.hip);
// this file routes a parsed chain to them.
//
//   k_init_generators: curand_init(seed_base + i, 0, 0) per state
//     (randInitKernel, src/utility_kernels.cuh:21-31).
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <type_traits>

#include "ikpso_device.h"
#include "ikpso_kernels.h"
#include "ikpso_swarm.h"
#include "ikpso_coop.h"
#include "ikpso_topo_ops.h"

namespace ikpso {

// ------------------------------------------------------------------ RNG init
__global__ void __launch_bounds__(256) k_init_generators(ikpso_rng_state* st, int64_t count, uint64_t seed_base)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < count;
         i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t s[6];
        xorwow_seed(seed_base + (uint64_t)i, s);
        ikpso_rng_state r;
        r.d = s[0];
        r.v[0] = s[1];
        r.v[1] = s[2];
        r.v[2] = s[3];
        r.v[3] = s[4];
        r.v[4] = s[5];
        r.boxmuller_flag = 0;
        r.boxmuller_flag_double = 0;
        r.boxmuller_extra = 0.0f;
        r.pad_ = 0;
        r.boxmuller_extra_double = 0.0;
        st[i] = r;
    }
}

// Seeds swarm-major states: state (b, i) = curand_init(seed_base + (first_swarm + b) * P + i).
// With a contiguous swarm range this is seed_base + first_swarm * P + flat index.
hipError_t launch_init_generators(ikpso_rng_state* st, int64_t count, uint64_t seed_base, hipStream_t stream)
{
    if (count <= 0) return hipSuccess;
    int64_t blocks = (count + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_init_generators, dim3((unsigned)blocks), dim3(256), 0, stream, st, count, seed_base);
    return hipGetLastError();
}

int resident_max_threads(const ChainHost& ch)
{
    int r = 0;
    visit_topology(ch, [&](auto topo) { r = kResidentMaxThreads<decltype(topo)::D>(); });
    return r;
}

bool chain_supported(const ChainHost& ch)
{
    return visit_topology(ch, [](auto) {});
}

std::string kernel_name(const ChainHost& ch, int family)
{
    const char* fam = family == IKPSO_KERNEL_COOP ? "swarm_coop" : family == IKPSO_KERNEL_STREAMING
                                                                       ? "swarm_streaming"
                                                                       : "swarm_resident";
    std::string topo = "generic";
    visit_topology(ch, [&](auto t) {
        using T = decltype(t);
        if constexpr (std::is_same_v<T, TopoRef7>)
            topo = "ref_tree7";
        else if constexpr (T::kDH)
            topo = "dh" + std::to_string(T::J);
        else if constexpr (!T::kGeneric)
            topo = "serial_tip" + std::to_string(T::J);
    });
    return std::string(fam) + "<" + topo + ">";
}

hipError_t launch_resident(const ChainHost& ch, int mode, const SwarmIO& io, hipStream_t stream)
{
    if (io.num_swarms <= 0) return hipSuccess;
    if (!ch.aux_dev) return hipErrorInvalidValue;  // the kernels read aux for the optional terms
    const int block = ((io.P + 63) / 64) * 64;
    hipError_t err = hipErrorInvalidValue;
    const bool ok = visit_topology(ch, [&](auto topo) {
        using T = decltype(topo);
        err = TopoOps<T>::resident(ch, mode, io, block, stream);
    });
    return ok ? err : hipErrorInvalidValue;
}

hipError_t launch_evaluate(const ChainHost& ch, int mode, const EvalIO& io, hipStream_t stream)
{
    if (io.n <= 0) return hipSuccess;
    if (!ch.aux_dev) return hipErrorInvalidValue;
    hipError_t err = hipErrorInvalidValue;
    const bool ok = visit_topology(ch, [&](auto topo) {
        using T = decltype(topo);
        err = TopoOps<T>::evaluate(ch, mode, io, stream);
    });
    return ok ? err : hipErrorInvalidValue;
}

hipError_t launch_coop(const ChainHost& ch, int mode, const SwarmIO& io, hipStream_t stream)
{
    if (io.num_swarms <= 0) return hipSuccess;
    if (!ch.aux_dev || io.coop_g <= 0 || io.coop_ng <= 0 || (!io.coop_linear && io.coop_ng % 8 != 0) ||
        !io.coop_slots || !io.coop_error)
        return hipErrorInvalidValue;
    hipError_t err = hipErrorInvalidValue;
    const bool ok = visit_topology(ch, [&](auto topo) {
        using T = decltype(topo);
        if (io.coop_g * kCoopThreads<T::D>() < io.P || io.coop_g > 64) return;  // G chunks must cover the swarm
        err = TopoOps<T>::coop(ch, mode, io, stream);
    });
    return ok ? err : hipErrorInvalidValue;
}

// Cooperative workgroups per CU: one for short chains (the kernel's LDS block is
// at least 82 KiB, more than half of a CU's 160 KiB), two for long ones
// (kCoopBlocksPerCU).
bool coop_geometry(const ChainHost& ch, int mode, CoopGeometry* g)
{
    (void)mode;
    bool spec = false;
    visit_topology(ch, [&](auto topo) {
        using T = decltype(topo);
        if constexpr (!T::kGeneric) {
            g->threads = kCoopThreads<T::D>();
            // the collider builds (which also carry the wide-angle chains, poly_trig) are
            // compiled for one workgroup per CU (kCoopMinWaves): plan for that residency,
            // or the launch could not fit the plan's groups
            g->blocks_per_cu = (ch.num_coll > 0 || ch.poly_trig) ? 1 : kCoopBlocksPerCU<T::D>();
            g->latency_variant = kCoopThreads<T::D>() != kCoopLatencyThreads;
            spec = true;
        }
    });
    if (!spec) return false;
    // the CU count, once per device (the plan runs on every latency-bound call)
    static std::mutex mu;
    static int c_dev = -1, c_cus = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    std::lock_guard<std::mutex> lk(mu);
    if (dev != c_dev) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return false;
        c_dev = dev, c_cus = cus;
    }
    g->cus = c_cus;
    return true;
}

// The latency variant of this chain runs with its generators on separate waves
// (k_swarm_coop_split: D <= 21, no mask, no collider block, hardware sin/cos range).
bool coop_latency_split(const ChainHost& ch)
{
    bool split = false;
    visit_topology(ch, [&](auto topo) {
        using T = decltype(topo);
        if constexpr (!T::kGeneric && kCoopThreads<T::D>() != kCoopLatencyThreads)
            split = IKPSO_SPLIT_GEN && T::D <= 21 && (T::kDH || !ch.masked) && ch.num_coll == 0 && !ch.poly_trig;
    });
    return split;
}

size_t coop_workspace_bytes(int ng, int G, int D, int block)
{
    return 8 * (size_t)ng * 2 * G * kCoopSlot(D) +
           256 + 3 * 256 + (IKPSO_COOP_TIMING ? 64 * (size_t)ng * G + 256 : 0);
}

hipError_t launch_stream(const ChainHost& ch, int mode, const StreamIO& io, int iterations, hipStream_t stream)
{
    if (io.num_swarms <= 0) return hipSuccess;
    if (!ch.aux_dev || io.C != (io.P + kStreamChunk - 1) / kStreamChunk) return hipErrorInvalidValue;
    hipError_t err = hipErrorInvalidValue;
    const bool ok = visit_topology(ch, [&](auto topo) {
        using T = decltype(topo);
        err = TopoOps<T>::stream(ch, mode, io, iterations, stream);
    });
    return ok ? err : hipErrorInvalidValue;
}

// Workspace bytes for B swarms of P particles and D angles (state excluded when
// the caller provides it).
size_t stream_workspace_bytes(int64_t B, int P, int D, bool with_state)
{
    const int64_t C = (P + kStreamChunk - 1) / kStreamChunk;
    size_t n = 0;
    if (with_state) n += sizeof(float) * (size_t)B * 3 * D * P + sizeof(float) * (size_t)B * P;
    n += sizeof(uint32_t) * 6 * (size_t)B * P;           // rng SoA
    n += (sizeof(uint32_t) + sizeof(int32_t)) * 2 * B * C;  // partial keys/idx
    n += sizeof(float) * 2 * B * C * D;                   // partial vectors
    n += (sizeof(uint32_t) + sizeof(int32_t)) * 2 * B;      // global best key/idx
    n += sizeof(float) * 2 * B * D;                       // global best vector
    return n + 8 * 256;                                   // alignment slack
}


}  // namespace ikpso
