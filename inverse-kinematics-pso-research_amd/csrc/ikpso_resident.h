// ikpso_resident.h -- the resident swarm kernel and the evaluate kernel
// (templates; instantiated per topology in ikpso_inst_*.hip).
//
//   k_swarm_resident: one workgroup = one swarm, one lane = one particle
//     (P <= 1024).  Position, velocity, local best, local-best fitness and the
//     XORWOW state of a particle stay on chip for all iterations; the chain
//     constants sit in the kernarg segment (scalar loads); the swarm argmin is
//     a DPP wave64 min + ballot, then one 16-entry LDS pass; the global-best
//     vector is broadcast through LDS only when it strictly improves (the
//     `globalMin > currentGlobalMin` test of src/kernel.cu:318).  HBM traffic
//     is the RNG state in/out and the outputs: the kernel is VALU-bound.
//
//   k_evaluate: FK + fitness of given angle vectors (parity/KAT entry).
#pragma once

#include <hip/hip_runtime.h>

#include "ikpso_device.h"
#include "ikpso_kernels.h"
#include "ikpso_swarm.h"

namespace ikpso {

// Chains of up to this many dimensions run 4 waves per SIMD (1024-lane
// workgroups) and take the software-pipelined FAST step (swarm_step_ahead);
// longer ones run 2 waves per SIMD, where the extra live node spills (3x slower).
constexpr int kTrigAheadMaxD = 30;
// Progress-levelled wave priority (progress_prio): levels of the 2-wave steps
// and of the pipelined 4-wave step.  Measured: config 5 81.1 -> 77.4 ms on 2048
// swarms x 100 iterations with 4 levels (profiles/r02c, r02d variant_timings);
// with two chunks of different swarms per CU (round 3) 3 levels are better:
// 4 / 3 / 2 / none 61.2 / 60.2 / 61.9 / 67.2 ms (profiles/r03s); config 3 48.3
// -> 47.3 ms with 2 levels, 51.7 ms with 4 (profiles/r02g); the folded DH arm's
// 4-wave tip-backward step unchanged within noise (so none).
#ifndef IKPSO_PRIO_LEVELS_2WAVE
#define IKPSO_PRIO_LEVELS_2WAVE 3
#endif
constexpr int kPrioLevels2Wave = IKPSO_PRIO_LEVELS_2WAVE, kPrioLevels4Wave = 2;

// Progress-levelled wave priority: entering node k of J a wave sets its issue
// priority to (L-1) - L(k-1)/J, so a wave that has run ahead of the others on
// its SIMD yields issue slots to the ones behind it.  The waves of a workgroup meet
// at the swarm argmin's barrier every iteration; under the arbiter's
// oldest-first tie-break the oldest wave finishes its step first and the last
// one runs its tail alone, with nothing to hide its dependency latency.
// With 4 waves per SIMD, 2 levels (4 keep them in lockstep, contending for the
// same unit at the same time).
// INV: the other way round -- a wave later in its step ranks higher.  The
// long-chain cooperative kernel (config 5) holds two workgroups of DIFFERENT
// swarms per CU, one wave of each per SIMD; ranked by progress they lock in
// phase and reach their exchanges together, leaving the SIMD idle while both
// wait.  Ranked the other way the one ahead finishes its step first and hands
// off while the other computes: 58.1 -> 57.1 ms on 2048 swarms x 4096 x 100,
// 232.6 -> 228.5 ms on 8192 (profiles/r04/variant_timings/var_c5inv*.txt; 2
// levels inverted: 60.7 ms, 4: 57.1 ms).
template <int J, int L, bool INV = false>
__device__ __forceinline__ void progress_prio(int k)
{
    static_assert(L == 0 || (L >= 2 && L <= 4), "priority levels: none or 2..4");
    if constexpr (L > 0) {
        switch (INV ? (L * (k - 1)) / J : (L - 1) - (L * (k - 1)) / J) {
        case 3: __builtin_amdgcn_s_setprio(3); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        default: __builtin_amdgcn_s_setprio(0); break;
        }
    }
}

// One PSO iteration of one particle (lane `tid`) of a swarm whose local bests
// sit in LDS as s_pb[d * BLOCK + lane] (shared by the resident and cooperative
// kernels).  simulateParticlesKernel (src/kernel.cu:153-189) + calculateDistance
// (src/kernel.cu:64-151), one node at a time: the node's three angles
// are updated (r1, r2, r3 per dimension, in dimension order) and
// clamped, then the node is folded into the FK/fitness.  A node's FK
// needs only its own and its ancestors' angles, so this computes the
// reference's update-all-then-evaluate values in the same order.  The
// node's LDS operands (local best, global best, rest pose, target) are
// loaded one node ahead so their latency hides under the previous node.
// simulateParticlesKernel for node k's A angles (draws r1, r2, r3 per
// dimension, in dimension order; then the clamp).
template <class Topo, int MODE, int TERMS, int BLOCK, class Rng>
__device__ __forceinline__ void update_node(const ChainConsts<Topo::J>& cc, const SwarmShared<Topo>& sh,
                                            const float* s_pb, int tid, int k, float (&x)[Topo::D],
                                            float (&v)[Topo::D], const PsoCoef& coef, Rng& rng)
{
    constexpr int A = Topo::A;
#pragma unroll
    for (int ax = 0; ax < A; ++ax) {
        const int d = A * (k - 1) + ax;
        if (kMasked<Topo, TERMS> && !dim_free(cc, d)) continue;  // locked: stays at rest
        pso_update<MODE>(x[d], v[d], s_pb[d * BLOCK + tid], sh.g[d], coef, rng);
        if constexpr (TERMS & kTermUniformBounds)
            x[d] = clamp_mode<MODE, true>(x[d], uniform_lo<TERMS>(cc), uniform_hi<TERMS>(cc));
        else
            x[d] = clamp_mode<MODE>(x[d], sh.lo[d], sh.hi[d]);
    }
}

// FAST: the same iteration software-pipelined by one node -- block k updates
// node k+1's angles and evaluates their sines and cosines while it folds node k
// into the FK, so the transcendental (or polynomial) latency of one node hides
// under another node's FK.  The draws keep dimension order.
template <class Topo, int MODE, int TERMS, int BLOCK, class Rng>
__device__ __forceinline__ float swarm_step_ahead(const ChainConsts<Topo::J>& cc, SwarmShared<Topo>& sh,
                                                  float* s_pb, int tid, float (&x)[Topo::D], float (&v)[Topo::D],
                                                  const PsoCoef& coef, Rng& rng)
{
    constexpr int J = Topo::J, A = Topo::A;
    constexpr int HW = kHwTrig<Topo, MODE, TERMS>;
    CandBuf<Topo, TERMS> cb;
    FitnessFor<Topo, MODE, TERMS> acc(cc, sh.dh, sh.soft, cb.v);
    progress_prio<J, kPrioLevels4Wave>(1);
    update_node<Topo, MODE, TERMS, BLOCK>(cc, sh, s_pb, tid, 1, x, v, coef, rng);
    NodeTrig<A> cur = node_trig<HW, A>(x);
#pragma unroll
    for (int k = 1; k <= J; ++k) {
        if (k > 1) progress_prio<J, kPrioLevels4Wave>(k);
        NodeTrig<A> nxt = cur;
        if (k < J) {
            update_node<Topo, MODE, TERMS, BLOCK>(cc, sh, s_pb, tid, k + 1, x, v, coef, rng);
            nxt = node_trig<HW, A>(x + A * k);
        }
        float rest[A], tgt[3];
#pragma unroll
        for (int ax = 0; ax < A; ++ax) rest[ax] = sh.rest[A * (k - 1) + ax];
#pragma unroll
        for (int c = 0; c < 3; ++c) tgt[c] = Topo::effector(k) ? sh.tgt[3 * (k - 1) + c] : 0.0f;
        acc.node_trig(cc, k, x + A * (k - 1), cur, rest, tgt, nullptr);
        cur = nxt;
        if (!Topo::kDH) __builtin_amdgcn_sched_barrier(0);
    }
    return acc.finish(cc);
}

// Serial chains with a tip effector and the folded chain (kTipBackward
// builds): all J nodes are updated in dimension order (the same draws; the
// angle terms in node order), then the tip is evaluated from the tip back
// (TipAccFor), each node's sines and cosines computed one node ahead of its
// rotation.  INV: the inverted wave priority (progress_prio), for the builds
// whose CU holds workgroups of two different swarms.
template <class Topo, int MODE, int TERMS, int BLOCK, int KA = 0, bool INV = false, class Rng>
__device__ __forceinline__ void swarm_step_tip(const ChainConsts<Topo::J>& cc, SwarmShared<Topo>& sh, float* s_pb,
                                               int tid, float (&x)[Topo::D], float (&v)[Topo::D], float& pbf,
                                               const PsoCoef& coef, Rng& rng, const float* pa = nullptr,
                                               const float* pc = nullptr)
{
    constexpr int J = Topo::J, A = Topo::A, D = Topo::D;
    constexpr int PL = D > kTrigAheadMaxD ? kPrioLevels2Wave : 0;  // wave priority: the 2-wave kernels
    using Acc = TipAccFor<Topo, MODE, TERMS>;
    Acc acc(sh.dh, sh.soft);
    float npb[A], ng[A], nrest[A];
#pragma unroll
    for (int ax = 0; ax < A; ++ax) {
        npb[ax] = s_pb[ax * BLOCK + tid];
        ng[ax] = sh.g[ax];
        nrest[ax] = sh.rest[ax];
    }
#pragma unroll
    for (int k = 1; k <= J; ++k) {
        progress_prio<2 * J, PL, INV>(k);
        float cpb[A], cg[A], crest[A];
#pragma unroll
        for (int ax = 0; ax < A; ++ax) {
            cpb[ax] = npb[ax];
            cg[ax] = ng[ax];
            crest[ax] = nrest[ax];
        }
        if (k < J) {
#pragma unroll
            for (int ax = 0; ax < A; ++ax) {
                const int d = A * k + ax;
                npb[ax] = s_pb[d * BLOCK + tid];
                ng[ax] = sh.g[d];
                nrest[ax] = sh.rest[d];
            }
        }
#pragma unroll
        for (int ax = 0; ax < A; ++ax) {
            const int d = A * (k - 1) + ax;
            if (d < KA)  // drawn ahead during the previous exchange (k_swarm_coop)
                pso_update_ahead(x[d], v[d], cg[ax], pa[d], pc[d]);
            else
                pso_update<MODE, true>(x[d], v[d], cpb[ax], cg[ax], coef, rng);
            if constexpr (TERMS & kTermUniformBounds)
                x[d] = clamp_mode<MODE, true>(x[d], uniform_lo<TERMS>(cc), uniform_hi<TERMS>(cc));
            else
                x[d] = clamp_mode<MODE>(x[d], sh.lo[d], sh.hi[d]);
        }
        acc.angles(k, x + A * (k - 1), crest);
        __builtin_amdgcn_sched_barrier(0);
    }
    NodeTrig<A> cur = node_trig<Acc::HW, A>(x + A * (J - 1));
#pragma unroll
    for (int k = J; k >= 1; --k) {
        progress_prio<2 * J, PL, INV>(2 * J + 1 - k);
        NodeTrig<A> nxt = cur;
        if (k > 1) nxt = node_trig<Acc::HW, A>(x + A * (k - 2));
        acc.back(cc, k, cur);
        cur = nxt;
        // (the folded chain's constants are LDS reads: left free to be issued ahead)
        if (!Topo::kDH) __builtin_amdgcn_sched_barrier(0);
    }
    float tgt[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) tgt[c] = sh.tgt[3 * (J - 1) + c];
    // updateLocalBests (src/kernel.cu:202-221): strict improvement
    const float f = acc.finish(cc, tgt);
    if (f < pbf) {
        pbf = f;
#pragma unroll
        for (int d = 0; d < D; ++d) s_pb[d * BLOCK + tid] = x[d];
    }
}

// Velocities the resident collider builds keep in LDS, behind the local bests
// (dimensions 0..kVelLds-1; the rest stay in registers).  node_collides is an
// out-of-line call (FitnessAcc::finish), and every value live across it that does
// not fit the callee-saved registers goes to scratch -- around the call and,
// through the register allocator's choices, on the main path, where a reload of a
// value spilled an iteration ago comes from HBM.  The velocities are read and
// written once per iteration: two LDS instructions per dimension.  Round 5, the
// collide leg's scene (4096 x 1024 x 500): 273 -> 222 ms, and 159 -> 102 ms with
// the boxes out of reach (profiles/r05/variant_timings/collide_cmp.txt).  The
// separating-axis builds have no call left (round 6): at most kVelLdsSat of them in
// LDS, the rest in registers without a spill -- 66.3 -> 65.2 ms on the collide leg
// (18 in LDS vs 9; 6 and 12 within 0.3 ms; profiles/r06/collcmp_near_variants.txt).
// The REFERENCE collider builds keep them all in LDS (9 spilled 21 registers there).
constexpr int kVelLdsSat = 9;
template <class Topo, int MODE, int TERMS>
__host__ __device__ constexpr int kVelLds()
{
    constexpr int D = Topo::D, BLOCK = kResidentMaxThreads<D>();
    if (!(TERMS & kTermColliders) || D > 30) return 0;
    constexpr long spare = 163840L - (long)sizeof(SwarmShared<Topo>) - 256 - (long)D * BLOCK * 4;
    constexpr long k = spare / (BLOCK * 4);
    constexpr int fit = k <= 0 ? 0 : (k >= D ? D : (int)k);
    return kFastSat<Topo, MODE, TERMS> && fit > kVelLdsSat ? kVelLdsSat : fit;
}

// The collider builds' call (node_collides, out of line in FitnessAcc::finish) may
// clobber SGPRs, so the chain constants the iteration keeps in SGPRs (loaded once
// from the kernel arguments) are parked in VGPR lanes across it and read back with
// v_readlane_b32 on the main path: 225 per iteration (round 5).  Re-reading them from
// the kernarg segment every iteration instead -- through a pointer the compiler
// cannot see is loop-invariant -- makes them scalar loads at their point of use.
#ifndef IKPSO_COLLIDE_RELOAD
#define IKPSO_COLLIDE_RELOAD 1
#endif
template <int J>
__device__ __forceinline__ const ChainConsts<J>& kernarg_cc()
{
    // the chain constants are the kernels' first argument: offset 0 of the kernarg segment
    const __attribute__((address_space(4))) char* p =
        (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const ChainConsts<J>*)(const char*)p;
}

// Masked chains (kMasked builds): a locked dimension takes no draws and keeps
// its rest value, as in the oracle's masked restatement.
// KV: velocities held in LDS behind the local bests (kVelLds; the resident kernel)
template <class Topo, int MODE, int TERMS, int BLOCK, int KV = 0, class Rng>
__device__ __forceinline__ void swarm_step(const ChainConsts<Topo::J>& cc, SwarmShared<Topo>& sh, float* s_pb,
                                           int tid, float (&x)[Topo::D], float (&v)[Topo::D], float& pbf,
                                           const PsoCoef& coef, Rng& rng)
{
    constexpr int J = Topo::J, A = Topo::A, D = Topo::D;
    constexpr bool MASK = kMasked<Topo, TERMS>;
    if constexpr (kTipBackward<Topo, MODE, TERMS>) {
        swarm_step_tip<Topo, MODE, TERMS, BLOCK>(cc, sh, s_pb, tid, x, v, pbf, coef, rng);
        return;
    }
    // (not the collider builds: the pipelined step's extra live node spilled them)
    if constexpr (MODE == IKPSO_ARITH_FAST && Topo::D <= kTrigAheadMaxD && !(TERMS & kTermColliders)) {
        // updateLocalBests (src/kernel.cu:202-221): strict improvement
        const float f = swarm_step_ahead<Topo, MODE, TERMS, BLOCK>(cc, sh, s_pb, tid, x, v, coef, rng);
        if (f < pbf) {
            pbf = f;
#pragma unroll
            for (int d = 0; d < D; ++d) s_pb[d * BLOCK + tid] = x[d];
        }
        return;
    }
    CandBuf<Topo, TERMS> cb;
    FitnessFor<Topo, MODE, TERMS> acc(cc, sh.dh, sh.soft, cb.v);
    if constexpr ((TERMS & kTermColliders) && SwarmShared<Topo>::kNear > 0 && !IKPSO_COLLIDE_STATS)
        acc.nearc = sh.near4;  // (the counting builds count through near_collider)
    float* const s_v = s_pb + D * BLOCK;  // KV > 0: velocities [d][lane] (kVelLds)
    // node kk's local bests, global best, rest angles, target and LDS velocities
    auto load_node = [&](int kk, float (&pb)[A], float (&g)[A], float (&rest)[A], float (&tgt)[3], float (&vv)[A]) {
#pragma unroll
        for (int ax = 0; ax < A; ++ax) {
            const int d = A * (kk - 1) + ax;
            pb[ax] = s_pb[d * BLOCK + tid];
            g[ax] = sh.g[d];
            rest[ax] = sh.rest[d];
            if (d < KV) vv[ax] = s_v[d * BLOCK + tid];
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) tgt[c] = Topo::effector(kk) ? sh.tgt[3 * (kk - 1) + c] : 0.0f;
    };
    // node k+1's LDS operands are read during node k (also in the collider builds,
    // where they are live across node_collides' call: reading them at node k instead
    // measured slower, 181 -> 209 ms with the boxes out of reach)
    float npb[A], ng[A], nrest[A], ntgt[3], nv[A];
    load_node(1, npb, ng, nrest, ntgt, nv);
#pragma unroll
    for (int k = 1; k <= J; ++k) {
        // the 2-wave kernels, and the 4-wave ones (D <= 30: only REFERENCE arithmetic takes
        // this path, FAST takes swarm_step_ahead): 2 levels, 16.98 -> 15.85 ms on the
        // REFERENCE resident kernel, config-3 shape (2048 x 1024 x 200,
        // profiles/r04/variant_timings/var_refprio.txt; 3 levels 15.89).  The cooperative
        // REFERENCE kernels (k_swarm_coop, k_swarm_coop_split) share this step and so the
        // levelling; they are the parity path and were not timed with and without it.
        progress_prio<J, (D > kTrigAheadMaxD ? kPrioLevels2Wave : kPrioLevels4Wave)>(k);
        float cpb[A], cg[A], crest[A], ctgt[3], cv[A];
#pragma unroll
        for (int ax = 0; ax < A; ++ax) {
            cpb[ax] = npb[ax];
            cg[ax] = ng[ax];
            crest[ax] = nrest[ax];
            if (A * (k - 1) + ax < KV) cv[ax] = nv[ax];
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) ctgt[c] = ntgt[c];
        if (k < J) load_node(k + 1, npb, ng, nrest, ntgt, nv);
#pragma unroll
        for (int ax = 0; ax < A; ++ax) {
            const int d = A * (k - 1) + ax;
            if (MASK && !dim_free(cc, d)) continue;  // locked: stays at rest
            if (d < KV) {
                pso_update<MODE>(x[d], cv[ax], cpb[ax], cg[ax], coef, rng);
                s_v[d * BLOCK + tid] = cv[ax];
            } else {
                pso_update<MODE>(x[d], v[d], cpb[ax], cg[ax], coef, rng);
            }
            if constexpr (TERMS & kTermUniformBounds)
                x[d] = clamp_mode<MODE, true>(x[d], uniform_lo<TERMS>(cc), uniform_hi<TERMS>(cc));
            else
                x[d] = clamp_mode<MODE>(x[d], sh.lo[d], sh.hi[d]);
        }
        acc.node(cc, k, x + A * (k - 1), crest, ctgt, nullptr);
        if (!Topo::kDH) __builtin_amdgcn_sched_barrier(0);
    }

    // updateLocalBests (src/kernel.cu:202-221): strict improvement
    const float f = acc.finish_for_update(cc, pbf);
    if (f < pbf) {
        pbf = f;
#pragma unroll
        for (int d = 0; d < D; ++d) s_pb[d * BLOCK + tid] = x[d];
    }
}

// initParticlesKernel (src/kernel.cu:223-266) for one particle: warm start at
// the current pose, v = U*2-1 (one draw per free dimension, in dimension
// order), local best = x.
template <class Topo, int TERMS, int BLOCK, class Rng>
__device__ __forceinline__ void init_particle(const ChainConsts<Topo::J>& cc, const SwarmShared<Topo>& sh,
                                              float* s_pb, int tid, float (&x)[Topo::D], float (&v)[Topo::D],
                                              Rng& rng)
{
#pragma unroll
    for (int d = 0; d < Topo::D; ++d) {
        x[d] = sh.rest[d];
        if (kMasked<Topo, TERMS> && !dim_free(cc, d))
            v[d] = 0.0f;
        else if constexpr (TERMS & kTermRev)  // (U * 2 - 1) / 2pi
            v[d] = __builtin_fmaf(rng.uniform(), 0.318309886183790672f, -kInv2Pi);
        else
            v[d] = __builtin_fmaf(rng.uniform(), 2.0f, -1.0f);
        s_pb[d * BLOCK + tid] = x[d];
    }
}

// ------------------------------------------------------- resident swarm kernel
// The kernel body over its LDS: the per-swarm uniforms `sh` and the local-best
// positions s_pb[d * BLOCK + lane] (read once per iteration by the update,
// written on improvement; consecutive lanes hit consecutive banks).
template <class Topo, int MODE, int TERMS>
__device__ __forceinline__ void swarm_resident_body(const ChainConsts<Topo::J>& cc, const SwarmIO& io,
                                                    SwarmShared<Topo>& sh, float* const s_pb)
{
    constexpr int D = Topo::D;
    constexpr int BLOCK = kResidentMaxThreads<D>();
    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x;
    const int P = io.P;
    const bool active = tid < P;

    stage_swarm_inputs<Topo, TERMS>(cc, io.targets, io.start_pose, b, sh);

    RngFor<TERMS> rng{0, 0, 0, 0, 0, 0};
    if (active) load_rng(rng, io.rng + b * P + tid);
    __syncthreads();

    // initParticlesKernel (src/kernel.cu:223-266)
    float x[D], v[D];
    init_particle<Topo, TERMS, BLOCK>(cc, sh, s_pb, tid, x, v, rng);
    constexpr int KV = kVelLds<Topo, MODE, TERMS>();
    float* const s_v = s_pb + D * BLOCK;  // (kVelLds)
#pragma unroll
    for (int d = 0; d < KV; ++d) s_v[d * BLOCK + tid] = v[d];
    // initLocalBests (src/kernel.cu:191-200)
    float pbf = fitness<Topo, MODE, TERMS>(cc, x, sh.rest, sh.tgt, nullptr, sh.dh, sh.soft);

    // swarm argmin + unconditional first global-best copy (src/kernel.cu:297-304)
    int bidx;
    uint32_t gkey = swarm_argmin(sh, 0, active ? ordered_key(pbf) : 0xFFFFFFFFu, &bidx);
    copy_gbest<Topo, BLOCK>(sh, s_pb, bidx);
    __syncthreads();

    const PsoCoef coef = pso_coef(cc);
    for (int it = 0; it < io.iterations; ++it) {
        compiler_fence();
        if constexpr ((TERMS & kTermColliders) && IKPSO_COLLIDE_RELOAD) {
            // the chain constants re-read from the kernarg segment every iteration (kernarg_cc)
            const ChainConsts<Topo::J>& cci = kernarg_cc<Topo::J>();
            swarm_step<Topo, MODE, TERMS, BLOCK, KV>(cci, sh, s_pb, tid, x, v, pbf, pso_coef(cci), rng);
        } else {
            swarm_step<Topo, MODE, TERMS, BLOCK, KV>(cc, sh, s_pb, tid, x, v, pbf, coef, rng);
        }

        // thrust::min_element + `globalMin > currentGlobalMin` (src/kernel.cu:315-323)
        const uint32_t bmin = swarm_argmin(sh, (it + 1) & 1, active ? ordered_key(pbf) : 0xFFFFFFFFu, &bidx);
        if (bmin < gkey) {  // uniform across the workgroup
            gkey = bmin;
            copy_gbest<Topo, BLOCK>(sh, s_pb, bidx);
            __syncthreads();
        }
    }

    // outputs: Coordinates result (updateGlobalBestCoordsKernel) + fitness + residual
    compiler_fence();
    store_angles<Topo, TERMS>(cc, io.out_angles, b, tid, tid < D ? sh.g[tid] : 0.0f);
    if (tid == 0 && io.out_fitness) io.out_fitness[b] = key_to_float(gkey);
    if (io.out_residual && tid < 64) {
        float g[D];
#pragma unroll
        for (int d = 0; d < D; ++d) g[d] = sh.g[d];
        const float r = residual<Topo, MODE, TERMS>(cc, g, sh.tgt, sh.dh);
        if (tid == 0) io.out_residual[b] = r;
    }
    if (active) {
        store_rng(rng, io.rng + b * P + tid);
        if (io.dump_particles) {  // reference particles layout [3][D][P] per swarm
            float* base = io.dump_particles + b * (int64_t)3 * D * P;
#pragma unroll
            for (int d = 0; d < D; ++d) {
                base[(int64_t)d * P + tid] = radians<TERMS>(x[d]);
                base[(int64_t)(D + d) * P + tid] = radians<TERMS>(d < KV ? s_v[d * BLOCK + tid] : v[d]);
                base[(int64_t)(2 * D + d) * P + tid] = radians<TERMS>(s_pb[d * BLOCK + tid]);
            }
        }
        if (io.dump_bests) io.dump_bests[b * P + tid] = pbf;
    }
}


#ifndef IKPSO_COLLIDE_UNIFORM
#define IKPSO_COLLIDE_UNIFORM 1  // the reference scene with colliders: a uniform-bounds FAST build (79.2 -> 77.2 ms)
#endif

// Waves per SIMD the resident kernel is compiled for.  The folded chain's
// iteration is short (458 VALU instructions per wave-iteration at 7 free angles)
// and two barriers of the swarm argmin end it: compiled for 8 waves per SIMD
// (<= 64 VGPRs: x, v, the generator and a handful of FK temporaries; the
// spills fall outside the iteration loop but for 0-11 scratch accesses per
// iteration) two swarms share a CU and one's barrier waits hide under the
// other's step -- iiwa arm, 4096 targets x 1024 x 500: 22.86 -> 18.43 ms
// (9.17e10 -> 1.14e11 updates/s, profiles/r03a/variant_timings/var_dh7_waves.txt).
// The Euler chains need more than 64 VGPRs (x, v and the node frames): one
// 1024-lane workgroup per CU, 4 waves per SIMD.
template <class Topo>
constexpr int kResidentMinWaves = Topo::kDH ? 8 : 1;

template <class Topo, int MODE, int TERMS>
__global__ void __launch_bounds__(kResidentMaxThreads<Topo::D>(), kResidentMinWaves<Topo>)
    k_swarm_resident(const ChainConsts<Topo::J> cc, const SwarmIO io)
{
    // local bests [d][lane], then the collider builds' LDS velocities (kVelLds)
    constexpr int NPB = (Topo::D + kVelLds<Topo, MODE, TERMS>()) * kResidentMaxThreads<Topo::D>();
    if constexpr (Topo::kGeneric) {
        // generic trees keep two arrays: hipcc 7.2 miscompiles them over one
        // LDS object (an illegal flat-to-LDS check)
        __shared__ SwarmShared<Topo> sh;
        __shared__ float s_pb[NPB];
        swarm_resident_body<Topo, MODE, TERMS>(cc, io, sh, s_pb);
    } else {
        __shared__ SwarmLds<Topo, NPB> lds;  // uniforms below 64 KiB (SwarmLds)
        swarm_resident_body<Topo, MODE, TERMS>(cc, io, lds.sh, lds.pb);
    }
}

// ----------------------------------------------------------- evaluate kernel
// angles, rest: [n][dfree] over the free dimensions (locked ones at the chain's rest).
template <class Topo, int MODE, int TERMS>
__global__ void __launch_bounds__(256) k_evaluate(const ChainConsts<Topo::J> cc, EvalIO io)
{
    constexpr int J = Topo::J;
    constexpr int D = Topo::D;
    const int64_t DF = cc.dfree;
    for (int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; n < io.n;
         n += (int64_t)gridDim.x * blockDim.x) {
        float x[D], rest[D], tgt[3 * J], pos[3 * J];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const bool fr = dim_free(cc, d);
            const int64_t r = n * DF + dim_rank(cc, d);
            x[d] = fr ? io.angles[r] : cc.rest[d];
            rest[d] = io.rest && fr ? io.rest[r] : cc.rest[d];
        }
        if (io.targets) {
#pragma unroll
            for (int k = 1; k <= J; ++k) {
                const int s = cc.eff_slot[k];
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    tgt[3 * (k - 1) + c] = s >= 0 ? io.targets[(n * cc.num_eff + s) * 3 + c] : 0.0f;
            }
        } else {
#pragma unroll
            for (int d = 0; d < 3 * J; ++d) tgt[d] = cc.tgt0[d];
        }
        const float f = fitness<Topo, MODE, TERMS>(cc, x, rest, tgt, pos, nullptr, cc.aux + 4 * J);
        if (io.out_fitness) io.out_fitness[n] = f;
        if (io.out_positions) {
#pragma unroll
            for (int d = 0; d < 3 * J; ++d) io.out_positions[n * 3 * J + d] = pos[d];
        }
    }
}

// --------------------------------------------------------------- dispatch
template <class Topo, int MODE>
inline hipError_t run_resident(const ChainHost& ch, const SwarmIO& io, int block, hipStream_t stream)
{
    const ChainConsts<Topo::J> cc = make_consts<Topo::J>(ch);
    const dim3 grid((unsigned)io.num_swarms), threads(block);
    // Term specialisation (FitnessAcc): the two hot configurations -- the
    // reference scene (uniform clamp bounds, no optional term) and BASELINE
    // config 5 (uniform bounds + soft-limit penalty) -- get their own FAST
    // kernels; everything else (generic topologies, the distance term, every
    // REFERENCE-mode run) tests the terms at run time with the same arithmetic,
    // with the collider block compiled in only when the scene has colliders.
    // The specialised FAST builds (and every folded-chain build) keep their
    // angles in revolutions (kTermRev).
    const int terms = term_set(ch);
    hipError_t err = hipSuccess;
    if (dh_terms<Topo>(terms, &err, [&](auto t) {
            hipLaunchKernelGGL((k_swarm_resident<Topo, MODE, decltype(t)::value | kTermRev>), grid, threads, 0, stream,
                               cc, io);
            return hipGetLastError();
        }))
        return err;
    if constexpr (!Topo::kGeneric && !Topo::kDH && MODE == IKPSO_ARITH_FAST) {
        if constexpr (std::is_same_v<Topo, TopoRef7>) {  // the reference scene's [0, 2pi] limits
            if (terms == kTermUniformBounds && ch.unit_rev_bounds) {
                hipLaunchKernelGGL((k_swarm_resident<Topo, MODE, kTermUniformBounds | kFastRev | kFastUnitBounds>),
                                   grid, threads, 0, stream, cc, io);
                return hipGetLastError();
            }
        }
        if (terms == kTermUniformBounds) {
            hipLaunchKernelGGL((k_swarm_resident<Topo, MODE, kTermUniformBounds | kFastRev>), grid, threads, 0, stream,
                               cc, io);
            return hipGetLastError();
        }
        if constexpr (std::is_same_v<Topo, TopoRef7> && IKPSO_COLLIDE_UNIFORM) {
            // the reference scene with colliders (the bench's collide leg): no runtime term tests, the clamp
            // bounds uniform (the separating-axis builds: colliders that are rotations, angles in the unit's range)
            if (terms == (kTermUniformBounds | kTermColliders) && ch.num_coll > 0 && ch.coll_obb && !ch.poly_trig) {
                hipLaunchKernelGGL((k_swarm_resident<Topo, MODE, kTermUniformBounds | kTermColliders>), grid, threads, 0,
                                   stream, cc, io);
                return hipGetLastError();
            }
        }
        if constexpr (std::is_same_v<Topo, TopoSerialTip<20>>) {  // BASELINE config 5's symmetric soft limits
            if (terms == (kTermUniformBounds | kTermPenalty) && ch.sym_penalty) {
                hipLaunchKernelGGL(
                    (k_swarm_resident<Topo, MODE, kTermUniformBounds | kTermPenalty | kFastRev | kFastSymPenalty>),
                    grid, threads, 0, stream, cc, io);
                return hipGetLastError();
            }
        }
        if (terms == (kTermUniformBounds | kTermPenalty)) {
            hipLaunchKernelGGL((k_swarm_resident<Topo, MODE, kTermUniformBounds | kTermPenalty | kFastRev>), grid,
                               threads, 0, stream, cc, io);
            return hipGetLastError();
        }
    }
    // REFERENCE on the reference scene (the bit-exact path the bench's reference_arith leg and the
    // recorded-trajectory replay run): no runtime term tests, the median clamp for ordered bounds
    if constexpr (std::is_same_v<Topo, TopoRef7> && MODE == IKPSO_ARITH_REFERENCE && IKPSO_REF_UNIFORM_BUILD) {
        if (terms == kTermUniformBounds && ch.ordered_bounds) {
            hipLaunchKernelGGL((k_swarm_resident<Topo, MODE, kTermUniformBounds>), grid, threads, 0, stream, cc, io);
            return hipGetLastError();
        }
    }
    (void)terms;
    return with_runtime_terms<Topo>(ch, [&](auto t) {
        hipLaunchKernelGGL((k_swarm_resident<Topo, MODE, decltype(t)::value>), grid, threads, 0, stream, cc, io);
        return hipGetLastError();
    });
}

template <class Topo, int MODE>
inline hipError_t run_evaluate(const ChainHost& ch, const EvalIO& io, hipStream_t stream)
{
    if constexpr (Topo::kDH) {  // the solver evaluates through its Euler chain
        return hipErrorNotSupported;
    } else {
    const ChainConsts<Topo::J> cc = make_consts<Topo::J>(ch);
    int64_t blocks = (io.n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    // the mask only places the given angles (no PSO): the unmasked builds evaluate it -- but a chain whose
    // angles reach beyond the transcendental unit's range (poly_trig) is solved by the masked collider
    // builds for their polynomial sin/cos, and is evaluated by the same arithmetic
    if ((ch.poly_trig && IKPSO_COLLIDE_HW_TRIG) || (ch.num_coll > 0 && !ch.coll_obb))
        hipLaunchKernelGGL((k_evaluate<Topo, MODE, kTermRuntime | kTermColliders | kTermMask>), dim3((unsigned)blocks),
                           dim3(256), 0, stream, cc, io);
    else if (ch.num_coll > 0)
        hipLaunchKernelGGL((k_evaluate<Topo, MODE, kTermRuntime | kTermColliders>), dim3((unsigned)blocks), dim3(256),
                           0, stream, cc, io);
    else
        hipLaunchKernelGGL((k_evaluate<Topo, MODE, kTermRuntime>), dim3((unsigned)blocks), dim3(256), 0, stream, cc,
                           io);
    return hipGetLastError();
    }
}

}  // namespace ikpso
