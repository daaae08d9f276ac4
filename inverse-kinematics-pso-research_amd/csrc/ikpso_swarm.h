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
template <class Topo>
struct SwarmShared {
    static constexpr int D = Topo::D, J = Topo::J;
    float lo[D], hi[D];          // clamp bounds
    float rest[D];               // warm start + angle-term reference
    float tgt[3 * J];            // effector targets per node (k-1), 0 elsewhere
    float g[D];                  // global-best vector
    float dh[Topo::kDH ? 12 * J + 4 : 1];  // folded-chain constants (TopoDH)
    float soft[6 * J];           // soft joint limits [lo 3J | hi 3J] (penalty term): read every
                                 // iteration, so from LDS rather than the aux array in HBM
    // the collider builds' inline sphere test (near_collider_lds): the first kNearUnroll
    // colliders' centres and squared limits per node, {cx, cy, cz, lim} at
    // [16 (k - 1) + 4 i], read by one broadcast ds_read_b128 each (compiled chains of
    // <= 8 joints; the others read them from the aux array by scalar loads)
    static constexpr int kNear = (!Topo::kGeneric && !Topo::kDH && J <= 8) ? 4 * kNearUnroll * J : 0;
    alignas(16) float near4[kNear > 0 ? kNear : 4];
    uint32_t key[2][16];         // per-wave argmin, double-buffered by parity
    int32_t idx[2][16];
};

// A swarm kernel's whole LDS as one object, the uniforms first: LDS addresses
// below 64 KiB fit a ds_read's 16-bit offset field, so every broadcast read of
// a uniform (sh.g[d], sh.rest[d], ...) addresses off one zero register.  Two
// separate __shared__ arrays may be laid out local bests first, putting the
// uniforms above 64 KiB, where every such read first materialises its absolute
// address with a v_mov (40 per iteration on the reference scene, 98 at D = 60).
template <class Topo, int NPB, class Extra = char>
struct SwarmLds {
    SwarmShared<Topo> sh;
    Extra extra;
    float pb[NPB];  // local bests [d][lane] (the cooperative long-chain build: velocities)
};

// start_pose: [B][dfree] over the free dimensions (the chain's mask).
// kTermRev builds: the angles (rest pose, clamp and soft limits) in revolutions.
template <class Topo, int TERMS = 0>
__device__ __forceinline__ void stage_swarm_inputs(const ChainConsts<Topo::J>& cc, const float* targets,
                                                   const float* start_pose, int64_t b, SwarmShared<Topo>& sh)
{
    constexpr int D = Topo::D, J = Topo::J;
    constexpr float sc = (TERMS & kTermRev) ? kInv2Pi : 1.0f;
    const float* t = targets ? targets + b * (int64_t)cc.num_eff * 3 : nullptr;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
        sh.lo[d] = cc.lo[d] * sc;
        sh.hi[d] = cc.hi[d] * sc;
        sh.rest[d] = (start_pose && dim_free(cc, d) ? start_pose[b * cc.dfree + dim_rank(cc, d)] : cc.rest[d]) * sc;
    }
    if constexpr (kOriginFrame<Topo, TERMS>) {
        // targets moved into the origin's frame: t' = M0^T (t - p0) (root_frame_sc)
        const float* m = cc.m0;
        for (int k = threadIdx.x; k < J; k += blockDim.x) {
            const int s = cc.eff_slot[k + 1];
            float w[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) w[c] = (t ? (s >= 0 ? t[3 * s + c] : 0.0f) : cc.tgt0[3 * k + c]) - m[4 * c + 3];
#pragma unroll
            for (int c = 0; c < 3; ++c)
                sh.tgt[3 * k + c] = s >= 0 ? m[c] * w[0] + m[4 + c] * w[1] + m[8 + c] * w[2] : 0.0f;
        }
    } else {
        for (int n = threadIdx.x; n < 3 * J; n += blockDim.x) {
            const int s = cc.eff_slot[n / 3 + 1];
            sh.tgt[n] = t ? (s >= 0 ? t[3 * s + n % 3] : 0.0f) : cc.tgt0[n];
        }
    }
    if constexpr (Topo::kDH)
        for (int n = threadIdx.x; n < 12 * J + 4; n += blockDim.x) sh.dh[n] = cc.aux[cc.dh_off + n];
    if (cc.use_penalty)
        for (int n = threadIdx.x; n < 6 * J; n += blockDim.x) sh.soft[n] = cc.aux[4 * J + n] * sc;
    if constexpr ((TERMS & kTermColliders) && SwarmShared<Topo>::kNear > 0)
        for (int n = threadIdx.x; n < kNearUnroll * J; n += blockDim.x) {
            const int k = n / kNearUnroll, i = n % kNearUnroll;
            if (i < cc.num_coll) {
                sh.near4[4 * n + 0] = cc.coll[i].px;
                sh.near4[4 * n + 1] = cc.coll[i].py;
                sh.near4[4 * n + 2] = cc.coll[i].pz;
                sh.near4[4 * n + 3] = cc.coll_lim[k * cc.num_coll + i];
            }
        }
}

// An angle of the kernel's units in radians (kTermRev: revolutions * 2 pi).
template <int TERMS>
__device__ __forceinline__ float radians(float a)
{
    if constexpr (TERMS & kTermRev)
        return a * k2Pi;
    else
        return a;
}

// The swarm's answer over the free dimensions: out[b][dfree] from the kernel's
// D-vector g (every thread of the calling workgroup; lanes < D write).
// kTermRev builds: g in revolutions, scaled back to radians; an answer that lies
// inside the clamp bounds (in the staged revolution bounds, lo * 1/2pi .. hi * 1/2pi)
// is held inside them in radians too (a bound's round trip through revolutions may
// land an ulp out).  An answer outside them -- the start pose itself, which the
// reference never clamps (src/kernel.cu:223-266), winning every iteration -- is
// returned as it is, as the reference returns it.
template <class Topo, int TERMS = 0>
__device__ __forceinline__ void store_angles(const ChainConsts<Topo::J>& cc, float* out, int64_t b, int d, float g)
{
    if (d < Topo::D && dim_free(cc, d)) {
        if constexpr (TERMS & kTermRev) {
            const bool inside = g >= cc.lo[d] * kInv2Pi && g <= cc.hi[d] * kInv2Pi;
            g *= k2Pi;
            if (inside) g = fminf(fmaxf(g, cc.lo[d]), cc.hi[d]);
        }
        out[b * cc.dfree + dim_rank(cc, d)] = g;
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

template <class SH>
__device__ __forceinline__ uint32_t swarm_argmin(SH& sh, int par, uint32_t key, int* out_idx)
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
template <class Topo, int BLOCK>
__device__ __forceinline__ void copy_gbest(SwarmShared<Topo>& sh, const float* s_pb, int idx)
{
    constexpr int D = Topo::D;
    static_assert(D <= 64, "one wave copies the global best");
    if (wave_id() == 0) {
        const int lane = lane_id_here();
        if (lane < D) sh.g[lane] = s_pb[lane * BLOCK + idx];
    }
}

// Term set of a chain for the kernel specialisation (see FitnessAcc): a masked
// chain carries kTermMask, which only the masked runtime-term builds match.
inline int term_set(const ChainHost& ch)
{
    return (ch.use_posref ? kTermPosRef : 0) | (ch.use_penalty ? kTermPenalty : 0) |
           (ch.uniform_bounds ? kTermUniformBounds : 0) | (ch.num_coll > 0 || ch.poly_trig ? kTermColliders : 0) |
           (ch.masked ? kTermMask : 0);
}

// The folded chain's builds: FAST, bounds uniform or not, penalty or not (it has
// no distance, collider or mask term).  Returns false for another term set.
template <class Topo, class F>
inline bool dh_terms(int terms, hipError_t* err, F&& f)
{
    if constexpr (Topo::kDH) {
        switch (terms) {
        case kTermUniformBounds: *err = f(std::integral_constant<int, kTermUniformBounds>{}); return true;
        case kTermUniformBounds | kTermPenalty:
            *err = f(std::integral_constant<int, kTermUniformBounds | kTermPenalty>{});
            return true;
        case 0: *err = f(std::integral_constant<int, 0>{}); return true;
        case kTermPenalty: *err = f(std::integral_constant<int, kTermPenalty>{}); return true;
        default: break;
        }
    }
    (void)terms;
    (void)err;
    return false;
}

// Visit the runtime-term build for a chain: kTermRuntime plus the collider
// block and the axis mask when the chain has them (the folded chain has neither).
template <class Topo, class F>
inline hipError_t with_runtime_terms(const ChainHost& ch, F&& f)
{
    if constexpr (Topo::kDH) {  // every term set of a folded chain has its own build (dh_terms)
        return hipErrorNotSupported;
    } else {
        // the collider builds also carry chains with wide angle ranges (poly_trig:
        // polynomial sin/cos; an empty collider loop)
        const bool coll = ch.num_coll > 0 || ch.poly_trig;
        // (IKPSO_COLLIDE_HW_TRIG: the unmasked collider builds use the transcendental unit,
        // so a wide-angle chain takes the masked build, whose sin/cos is the polynomial)
        if (coll && (ch.masked || (IKPSO_COLLIDE_HW_TRIG && ch.poly_trig) || (ch.num_coll > 0 && !ch.coll_obb)))
            return f(std::integral_constant<int, kTermRuntime | kTermColliders | kTermMask>{});
        if (coll) return f(std::integral_constant<int, kTermRuntime | kTermColliders>{});
        if (ch.masked) return f(std::integral_constant<int, kTermRuntime | kTermMask>{});
        return f(std::integral_constant<int, kTermRuntime>{});
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
#if IKPSO_WITH_DH
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
    case TopoKind::DH:
        switch (ch.J) {  // free angles of a folded serial chain (DH arms: 3-12)
#if IKPSO_WITH_DH
#define IKPSO_D(n) \
    case n: f(TopoDH<n>{}); return true;
            IKPSO_D(3) IKPSO_D(4) IKPSO_D(5) IKPSO_D(6) IKPSO_D(7) IKPSO_D(8) IKPSO_D(9) IKPSO_D(10) IKPSO_D(11)
                IKPSO_D(12)
#undef IKPSO_D
#endif
        default: break;
        }
        return false;  // no generic fallback: the caller keeps the Euler chain
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
