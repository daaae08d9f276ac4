// ikpso_swarm.h -- device helpers shared by the resident and streaming swarm
// kernels: per-swarm LDS staging, the swarm argmin, generator state I/O, and
// the host-side dispatch over compiled topologies.
#pragma once

#include <hip/hip_runtime.h>

#include "ikpso_device.h"
#include "ikpso_kernels.h"

namespace ikpso {

template <class Rng>
__device__ __forceinline__ void load_rng(Rng& r, const ikpso_rng_state* p)
{
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
    r.d = q[0];
    r.v0 = q[1];
    r.v1 = q[2];
    r.v2 = q[3];
    r.v3 = q[4];
    r.v4 = q[5];
}

template <class Rng>
__device__ __forceinline__ void store_rng(const Rng& r, ikpso_rng_state* p)
{
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    q[0] = r.d;
    q[1] = r.v0;
    q[2] = r.v1;
    q[3] = r.v2;
    q[4] = r.v3;
    q[5] = r.v4;
}

// Per-swarm uniform constants staged in LDS.  They are read at their point of
// use every iteration (an empty asm with a memory clobber at the top of the
// iteration stops the compiler from hoisting them into registers): ~100
// loop-invariant uniforms held in SGPRs/VGPRs across the loop spill, while a
// broadcast ds_read costs one LDS cycle.
template <int J>
struct SwarmShared {
    float lo[3 * J], hi[3 * J];  // clamp bounds
    float rest[3 * J];           // warm start + angle-term reference
    float tgt[3 * J];            // effector targets per node (k-1), 0 elsewhere
    float g[3 * J];              // global-best vector
    uint32_t key[2][16];         // per-wave argmin, double-buffered by parity
    int32_t idx[2][16];
};

template <int J>
__device__ __forceinline__ void stage_swarm_inputs(const ChainConsts<J>& cc, const float* targets,
                                                   const float* start_pose, int64_t b, SwarmShared<J>& sh)
{
    constexpr int D = 3 * J;
    const float* t = targets ? targets + b * (int64_t)cc.num_eff * 3 : nullptr;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
        sh.lo[d] = cc.lo[d];
        sh.hi[d] = cc.hi[d];
        sh.rest[d] = start_pose ? start_pose[b * D + d] : cc.rest[d];
        const int s = cc.eff_slot[d / 3 + 1];
        sh.tgt[d] = t ? (s >= 0 ? t[3 * s + d % 3] : 0.0f) : cc.tgt0[d];
    }
}

__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

// One swarm's particle planes [3][D][P] (position | velocity | local best)
// through a buffer resource: the lane's offset lives in one VGPR and the
// per-dimension offset (plane*D + d) * P * 4 in an SGPR, instead of a 64-bit
// VGPR address per access (which the compiler otherwise precomputes and keeps
// live for every one of the 3D accesses).
struct Planes {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t p4;    // P * 4
    uint32_t voff;  // lane * 4
    int D;

    __device__ __forceinline__ Planes(float* swarm_base, int D_, int P, int i)
        : rsrc(__builtin_amdgcn_make_buffer_rsrc(swarm_base, 0, 3 * D_ * P * 4, 0x00020000)),
          p4((uint32_t)P * 4u), voff((uint32_t)i * 4u), D(D_)
    {
    }
    __device__ __forceinline__ float ld(int plane, int d) const
    {
        return __uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)voff, (int)((uint32_t)(plane * D + d) * p4), 0));
    }
    __device__ __forceinline__ void st(int plane, int d, float v) const
    {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc, (int)voff,
                                              (int)((uint32_t)(plane * D + d) * p4), 0);
    }
};

// Swarm argmin of the local-best fitness keys, lowest particle index on ties
// (thrust::min_element, src/kernel.cu:297,315).  One DPP wave min + ballot per
// wave, a 16-entry LDS exchange, then every wave reduces the 16 entries
// redundantly, so the result is uniform without a second barrier.  Everything
// after the wave min is scalar (wave id, first lane, winner index): the only
// per-lane value is the lane id from mbcnt, so nothing here needs threadIdx
// kept live across the loop (the compiler spilled it, and the reload sat on
// the barrier's critical path).
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Lane id recomputed at the point of use (two VALU ops): an opaque asm, so the
// compiler can neither hoist it out of the iteration loop nor keep it live
// (and spill it) across the loop body.
__device__ __forceinline__ int lane_id_here()
{
    int lane;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    return lane;
}

template <int J>
__device__ __forceinline__ uint32_t swarm_argmin(SwarmShared<J>& sh, int par, uint32_t key, int* out_idx)
{
    const int lane = lane_id_here(), wave = wave_id();
    const int nwaves = blockDim.x >> 6;
    const uint32_t wmin = wave_min_u32(key);
    const int first = wave_first_lane_eq(key, wmin);
    if (lane == 0) {
        sh.key[par][wave] = wmin;
        sh.idx[par][wave] = wave * 64 + first;
    }
    __syncthreads();
    const uint32_t k2 = lane < nwaves ? sh.key[par][lane] : 0xFFFFFFFFu;
    const uint32_t bmin = wave_min_u32(k2);
    *out_idx = __builtin_amdgcn_readfirstlane(sh.idx[par][wave_first_lane_eq(k2, bmin)]);
    return bmin;
}

// sh.g = local best of particle `idx` (updateGlobalBestCoordsKernel,
// src/kernel.cu:268-277), copied by the first wave; the caller barriers.
template <int J, int BLOCK>
__device__ __forceinline__ void copy_gbest(SwarmShared<J>& sh, const float* s_pb, int idx)
{
    constexpr int D = 3 * J;
    static_assert(D <= 64, "one wave copies the global best");
    if (wave_id() == 0) {
        const int lane = lane_id_here();
        if (lane < D) sh.g[lane] = s_pb[lane * BLOCK + idx];
    }
}

// Visit the kernel instantiation for (topology, J, mode).  Returns false when
// the chain has no compiled variant.
template <class F>
inline bool visit_topology(const ChainHost& ch, F&& f)
{
    switch (ch.topo) {
    case TopoKind::Ref7:
#if IKPSO_WITH_REF7
        f(TopoRef7{});
        return true;
#else
        break;
#endif
    case TopoKind::SerialTip:
        switch (ch.J) {  // arm lengths of DH arms (6-14 nodes: 6-7 joints + d offsets) and BASELINE config 5
#if IKPSO_WITH_OTHERS
#define IKPSO_S(n) \
    case n: f(TopoSerialTip<n>{}); return true;
            IKPSO_S(6) IKPSO_S(7) IKPSO_S(8) IKPSO_S(9) IKPSO_S(10) IKPSO_S(11) IKPSO_S(12) IKPSO_S(13) IKPSO_S(14)
#undef IKPSO_S
#endif
#if IKPSO_WITH_SERIAL20
        case 20: f(TopoSerialTip<20>{}); return true;
#endif
        default: break;
        }
        break;
    case TopoKind::Generic:
        break;
    }
#if IKPSO_WITH_OTHERS
    switch (ch.J) {  // any tree: runtime parent indices
#define IKPSO_G(n) \
    case n: f(TopoGeneric<n>{}); return true;
        IKPSO_G(1) IKPSO_G(2) IKPSO_G(3) IKPSO_G(4) IKPSO_G(5) IKPSO_G(6) IKPSO_G(7) IKPSO_G(8) IKPSO_G(9)
            IKPSO_G(10) IKPSO_G(11) IKPSO_G(12) IKPSO_G(13) IKPSO_G(14) IKPSO_G(15) IKPSO_G(16) IKPSO_G(17)
                IKPSO_G(18) IKPSO_G(19) IKPSO_G(20)
#undef IKPSO_G
    default: break;
    }
#endif
    return false;
}


}  // namespace ikpso
