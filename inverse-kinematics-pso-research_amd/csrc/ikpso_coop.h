// ikpso_coop.h -- cooperative resident swarm kernel: one swarm spread over G
// co-resident workgroups (G CUs), state on chip for the whole solve.
//
// For swarms larger than one workgroup (BASELINE config 5: 4096 particles of a
// 60-angle chain; the visualiser's N = 16384) the streaming kernels move
// x, v and the local bests through HBM every iteration (12·D bytes per
// particle-update: HBM-bound).  Here every workgroup keeps its chunk of
// BLOCK particles resident exactly as k_swarm_resident does (x, v, generator
// state in VGPRs, local bests in LDS) and the G chunks of a swarm meet once
// per iteration to form the swarm's argmin (thrust::min_element +
// `globalMin > currentGlobalMin`, src/kernel.cu:297-323):
//
//   each chunk: local argmin (first minimum) -> wave 0 publishes its record
//   for exchange e -- the key and the winner's local best, each value in an
//   8-byte granule {value, tag = e + 1} written by ONE `sc1` store (lane l
//   writes granule l) -> wave 0 polls the G key granules (lanes 0..G-1,
//   `global_load_dwordx2 sc1`) until every tag reads e + 1 -> reduces the G
//   keys in chunk order (ties keep the lowest chunk = lowest particle index)
//   -> on strict improvement takes the winner's vector (its own from LDS, or
//   the winner's D granules, re-polled until every tag reads e + 1) into LDS
//   -> workgroup barrier.
//
// This is MI355X_MICROARCH.md's tagged-granule hand-off (handoff-1to1: one
// hop, ~1 us; a separate flag or counter costs 1.7-1.9x that per hop, and the
// counter protocol this replaces chained four hops: ~12k cycles of a 31k-cycle
// iteration at D = 60).  A granule is written whole by one store and carries
// its own exchange number, so no store needs a vmcnt wait and no load needs a
// fence.  Records are double-buffered by exchange parity: a chunk rewrites
// parity p only after it has seen every chunk's record of the previous
// exchange, by which time every chunk has finished reading parity p.  The
// slots are zeroed before every launch (tag 0 never matches).  Workgroup b sits
// on XCD b % 8; the G chunks of a group share an XCD (speed only, never
// correctness).  Waits are bounded: a timed-out wait sets io.coop_error and
// the kernel drains.
// Residency is checked at launch against the occupancy query.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "ikpso_resident.h"

namespace ikpso {


// 8-byte granule access with agent scope: `global_store/load_dwordx2 sc1`
// (global, never flat: the pointer is cast to the global address space).
using granule_t = unsigned long long;
typedef __attribute__((address_space(1))) granule_t global_granule;
__device__ __forceinline__ void st_granule(granule_t* p, granule_t v)
{
    __hip_atomic_store((global_granule*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ granule_t ld_granule(const granule_t* p)
{
    return __hip_atomic_load((global_granule*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-workgroup bookkeeping in LDS, read at its points of use: held in SGPRs
// across the iteration loop it pushes the chain constants out of the scalar
// file and the resulting spills cost VGPRs (the resident kernel's rule, see
// SwarmShared).
template <int J>
struct CoopShared {
    uint32_t gkey;      // the swarm's global-best key (uniform copy for every wave)
    int32_t abort;      // a group wait timed out: drain
    int32_t G, member;  // chunks per swarm, this workgroup's chunk
    uint32_t e;         // exchanges of this group so far (identical in every member)
    int32_t pad_;
    int64_t b;          // current swarm
    granule_t* slots;   // the group's [2][G] published records (kCoopSlot granules each)
#if IKPSO_COOP_TIMING
    unsigned long long t_mid;  // wave 0 past the local argmin (timing builds)
#endif
};

// Exchange `e` of a group: publish this chunk's local argmin, wait for the G
// chunks, reduce; returns the group-wide minimum key of this exchange (uniform)
// and leaves the winner's local best in sh.g when it improves on `gkey` (or
// always when `force`).  Called by every wave; wave 0 does the global work.
// One chunk's local-best plane [d][lane] in global memory (coop_global_pbest):
// a buffer resource, so an access costs one VGPR offset (the lane) and an SGPR
// offset (the dimension) instead of a 64-bit address per dimension.
struct PbPlane {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t voff;
    __device__ __forceinline__ PbPlane(float* base, int D, int block, int lane)
        : rsrc(__builtin_amdgcn_make_buffer_rsrc(base, 0, D * block * 4, 0x00020000)), voff((uint32_t)lane * 4u)
    {
    }
    template <int BLOCK>
    __device__ __forceinline__ float ld(int d) const
    {
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)voff, d * BLOCK * 4, 0));
    }
    template <int BLOCK>
    __device__ __forceinline__ void st(int d, float v) const
    {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc, (int)voff, d * BLOCK * 4, 0);
    }
};

// The winner's local best: from the LDS array [d][lane] or the global plane.
template <int BLOCK>
__device__ __forceinline__ float local_best(const float* s_pb, int d, int lane)
{
    return s_pb[d * BLOCK + lane];
}
template <int BLOCK>
__device__ __forceinline__ float local_best(const PbPlane& pb, int d, int lane)
{
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pb.rsrc, lane * 4, d * BLOCK * 4, 0));
}

template <class Topo, int BLOCK, class PB>
__device__ __forceinline__ void coop_exchange(SwarmShared<Topo>& sh, CoopShared<Topo::J>& cs, const PB& s_pb,
                                              uint32_t local_key, int32_t* error, uint32_t spin_limit, bool force)
{
    constexpr int D = Topo::D;
    constexpr int SLOT = kCoopSlot(D);
    static_assert(D + 1 <= 64, "wave 0 publishes the record in one store instruction");
    int lidx;
    const uint32_t lmin = swarm_argmin(sh, 0, local_key, &lidx);  // one workgroup barrier inside
#if IKPSO_COOP_NO_EXCHANGE  // timing-only ablation: every chunk its own swarm (no cross-CU hand-off)
    if (wave_id() == 0) {
        const int lane = lane_id_here();
        if (force || lmin < cs.gkey) {
            if (lane < D) sh.g[lane] = local_best<BLOCK>(s_pb, lane, lidx);
            if (lane == 0) cs.gkey = lmin;
        }
        (void)error, (void)spin_limit, (void)SLOT;
    }
    __syncthreads();
    return;
#endif
    if (wave_id() == 0) {
        compiler_fence();
#if IKPSO_COOP_TIMING
        cs.t_mid = __builtin_amdgcn_s_memtime();
#endif
        const int G = cs.G, member = cs.member;
        const uint32_t e = cs.e;
        const int lane = lane_id_here();
        const granule_t tag = (granule_t)(e + 1) << 32;
        granule_t* base = cs.slots + (size_t)(e & 1) * G * SLOT;
        // granule 0: the key; granules 1..D: the chunk winner's local best
        const float mine_d = lane >= 1 && lane <= D ? local_best<BLOCK>(s_pb, lane - 1, lidx) : 0.0f;
        if (lane <= D) st_granule(base + (size_t)member * SLOT + lane, tag | (lane == 0 ? lmin : __float_as_uint(mine_d)));
        // the G key granules, in chunk order (lanes 0..G-1; G <= 64)
        uint32_t n = 0;
        int timed_out = 0;
        granule_t kg;
        for (;;) {
            kg = lane < G ? ld_granule(base + (size_t)lane * SLOT) : tag;
            if (__builtin_amdgcn_ballot_w64((kg >> 32) != (granule_t)(e + 1)) == 0) break;
            if (spin_limit == 0 || n++ >= spin_limit) {  // spin_limit 0 (IKPSO_COOP_SPIN_LIMIT=0): the give-up path
                timed_out = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const uint32_t k = lane < G ? (uint32_t)kg : 0xFFFFFFFFu;
        const uint32_t gmin = wave_min_u32(k);
        const int wj = wave_first_lane_eq(k, gmin);
        const uint32_t cur = cs.gkey;
        if (!timed_out && (force || gmin < cur)) {  // uniform within wave 0
            float gv = mine_d;  // this chunk won: its own vector, no hop
            if (wj != member) {
                granule_t vg;
                for (;;) {  // the winner's D granules (their tags already read e + 1 in practice)
                    vg = lane >= 1 && lane <= D ? ld_granule(base + (size_t)wj * SLOT + lane) : tag;
                    if (__builtin_amdgcn_ballot_w64((vg >> 32) != (granule_t)(e + 1)) == 0) break;
                    if (n++ >= spin_limit) {
                        timed_out = 1;
                        break;
                    }
                }
                gv = __uint_as_float((uint32_t)vg);
            }
            if (lane >= 1 && lane <= D) sh.g[lane - 1] = gv;
            if (lane == 0) cs.gkey = gmin;
        }
        if (lane == 0) {
            cs.e = e + 1;
            if (timed_out) {
                cs.abort = 1;
                __hip_atomic_store(error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    __syncthreads();
}

#ifndef IKPSO_COOP_SHL1_ADD
#define IKPSO_COOP_SHL1_ADD 0  // the add-for-shift generator form in the throughput build too
#endif
#ifndef IKPSO_PBG_HW
#define IKPSO_PBG_HW 1        // FAST sin/cos on the transcendental unit in the long-chain build
#endif
#ifndef IKPSO_PBG_AHEAD
#define IKPSO_PBG_AHEAD 2     // nodes of local bests loaded ahead of their use
#endif
#ifndef IKPSO_PBG_V_AHEAD
#define IKPSO_PBG_V_AHEAD 1   // nodes of velocities read from LDS ahead of their use
#endif

// One PSO iteration of the long-chain build: positions in VGPRs, velocities in
// LDS (s_v[d][lane]), local bests in the chunk's global plane, loaded
// IKPSO_PBG_AHEAD nodes ahead.  Same arithmetic and draw order as swarm_step.
template <class Topo, int MODE, int TERMS, int BLOCK, class Rng>
__device__ __forceinline__ void swarm_step_pbg(const ChainConsts<Topo::J>& cc, SwarmShared<Topo>& sh, float* s_v,
                                               const PbPlane& pb, int tid, float (&x)[Topo::D], float& pbf,
                                               const PsoCoef& coef, Rng& rng)
{
    constexpr int J = Topo::J, A = Topo::A, D = Topo::D;
    constexpr bool MASK = kMasked<Topo, TERMS>;
    constexpr bool HW = IKPSO_PBG_HW && IKPSO_SINCOS_HW && MODE == IKPSO_ARITH_FAST && !(TERMS & kTermColliders);
    constexpr int AH = (IKPSO_PBG_AHEAD < J) ? IKPSO_PBG_AHEAD : J;
    constexpr int VH = (IKPSO_PBG_V_AHEAD < J) ? IKPSO_PBG_V_AHEAD : J;
    FitnessFor<Topo, MODE, TERMS> acc(cc, sh.dh, sh.soft);
    float ring[AH + 1][A], vring[VH + 1][A];
#pragma unroll
    for (int n = 0; n < AH; ++n)
#pragma unroll
        for (int ax = 0; ax < A; ++ax) ring[n][ax] = pb.template ld<BLOCK>(A * n + ax);
#pragma unroll
    for (int n = 0; n < VH; ++n)
#pragma unroll
        for (int ax = 0; ax < A; ++ax) vring[n][ax] = s_v[(A * n + ax) * BLOCK + tid];
#pragma unroll
    for (int k = 1; k <= J; ++k) {
        const int cs = (k - 1) % (AH + 1), cv = (k - 1) % (VH + 1);
        float cpb[A], cvel[A];
#pragma unroll
        for (int ax = 0; ax < A; ++ax) {
            cpb[ax] = ring[cs][ax];
            cvel[ax] = vring[cv][ax];
        }
        if (k - 1 + AH < J) {
            const int nn = k - 1 + AH, ns = nn % (AH + 1);
#pragma unroll
            for (int ax = 0; ax < A; ++ax) ring[ns][ax] = pb.template ld<BLOCK>(A * nn + ax);
        }
        if (k - 1 + VH < J) {
            const int nn = k - 1 + VH, ns = nn % (VH + 1);
#pragma unroll
            for (int ax = 0; ax < A; ++ax) vring[ns][ax] = s_v[(A * nn + ax) * BLOCK + tid];
        }
#pragma unroll
        for (int ax = 0; ax < A; ++ax) {
            const int d = A * (k - 1) + ax;
            if (MASK && !dim_free(cc, d)) continue;  // locked: stays at rest
            float vv = cvel[ax];
            pso_update<MODE>(x[d], vv, cpb[ax], sh.g[d], coef, rng);
            s_v[d * BLOCK + tid] = vv;
            if constexpr (TERMS & kTermUniformBounds)
                x[d] = clamp_mode<MODE>(x[d], cc.lo[0], cc.hi[0]);
            else
                x[d] = clamp_mode<MODE>(x[d], sh.lo[d], sh.hi[d]);
        }
        float rest[A], tgt[3];
#pragma unroll
        for (int ax = 0; ax < A; ++ax) rest[ax] = sh.rest[A * (k - 1) + ax];
#pragma unroll
        for (int c = 0; c < 3; ++c) tgt[c] = Topo::effector(k) ? sh.tgt[3 * (k - 1) + c] : 0.0f;
        if constexpr (MODE == IKPSO_ARITH_FAST)
            acc.node_trig(cc, k, x + A * (k - 1), node_trig<HW, A>(x + A * (k - 1)), rest, tgt, nullptr);
        else
            acc.node(cc, k, x + A * (k - 1), rest, tgt, nullptr);
        __builtin_amdgcn_sched_barrier(0);
    }
    // updateLocalBests (src/kernel.cu:202-221): strict improvement
    const float f = acc.finish(cc);
    if (f < pbf) {
        pbf = f;
#pragma unroll
        for (int d = 0; d < D; ++d) pb.template st<BLOCK>(d, x[d]);
    }
}

// BLOCK: kCoopThreads<D>() (throughput: fill each CU), or kCoopLatencyThreads
// for a few swarms (latency: one wave per SIMD on 4x more CUs).
template <class Topo, int MODE, int TERMS, int BLOCK>
__global__ void __launch_bounds__(BLOCK, (BLOCK >= 256 ? BLOCK / 256 : 1))
    k_swarm_coop(const ChainConsts<Topo::J> cc, const SwarmIO io)
{
    constexpr int J = Topo::J;
    constexpr int D = Topo::D;
    constexpr bool PBG = coop_global_pbest(D);
    const int tid = threadIdx.x;
    const int P = io.P;

    // local bests [d][lane] (PBG: the velocities; the local bests are in the
    // chunk's global plane); padded to > 80 KiB so a CU never holds two
    // workgroups (the launch geometry assumes one per CU)
    constexpr int kPb = (D * BLOCK * 4 > 82 * 1024) ? D * BLOCK : 82 * 1024 / 4;
    __shared__ SwarmLds<Topo, kPb, CoopShared<J>> lds;
    SwarmShared<Topo>& sh = lds.sh;
    CoopShared<J>& cs = lds.extra;
    float* const s_pb = lds.pb;
    const PbPlane pbg(PBG ? io.coop_pbest + (size_t)blockIdx.x * D * BLOCK : nullptr, D, BLOCK, tid);
    if (tid == 0) {
        // XCD-aware group membership: workgroups b, b+8, b+16, ... share an XCD
        const int G = io.coop_g;
        const int xcd = blockIdx.x & 7, pos = blockIdx.x >> 3;
        const int group = (pos / G) * 8 + xcd;
        cs.G = G;
        cs.member = pos % G;
        cs.e = 0;
        cs.abort = 0;
        cs.b = group;
        cs.slots = io.coop_slots + (size_t)group * 2 * G * kCoopSlot(D);
    }
    __syncthreads();
    const PsoCoef coef = pso_coef(cc);

    for (;;) {
        compiler_fence();
        const int64_t b = cs.b;
        if (b >= io.num_swarms) break;
        const int i = cs.member * BLOCK + tid;  // particle index within the swarm
        stage_swarm_inputs<Topo>(cc, io.targets, io.start_pose, b, sh);
        // the add-for-shift issue form only in the latency variant (one wave per
        // SIMD, room to spare): in the 2-wave serial-20 kernel it cost 5 %
        using Rng = XorwowT<(IKPSO_COOP_SHL1_ADD || BLOCK == kCoopLatencyThreads) &&
                            std::is_same_v<RngFor<TERMS>, XorwowT<true>>>;
        Rng rng{0, 0, 0, 0, 0, 0};
        if (i < P) load_rng(rng, io.rng + b * P + i);
        if (tid == 0) cs.gkey = 0xFFFFFFFFu;
        __syncthreads();

        // initParticlesKernel + initLocalBests (src/kernel.cu:191-266)
        float x[D], v[PBG ? 1 : D];
        if constexpr (PBG) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                x[d] = sh.rest[d];
                const bool locked = kMasked<Topo, TERMS> && !dim_free(cc, d);
                s_pb[d * BLOCK + tid] = locked ? 0.0f : __builtin_fmaf(rng.uniform(), 2.0f, -1.0f);
                pbg.template st<BLOCK>(d, x[d]);
            }
        } else {
            init_particle<Topo, TERMS, BLOCK>(cc, sh, s_pb, tid, x, v, rng);
        }
        float pbf = fitness<Topo, MODE, TERMS>(cc, x, sh.rest, sh.tgt, nullptr, sh.dh, sh.soft);
        // swarm argmin + unconditional first global-best copy (src/kernel.cu:297-304)
        const uint32_t key0 = i < P ? ordered_key(pbf) : 0xFFFFFFFFu;
        if constexpr (PBG)
            coop_exchange<Topo, BLOCK>(sh, cs, pbg, key0, io.coop_error, io.coop_spin_limit, true);
        else
            coop_exchange<Topo, BLOCK>(sh, cs, s_pb, key0, io.coop_error, io.coop_spin_limit, true);

#if IKPSO_COOP_TIMING
        unsigned long long t_step = 0, t_bar = 0, t_exch = 0, n_it = 0;
#endif
        for (int it = 0; it < io.iterations; ++it) {
            compiler_fence();
            if (cs.abort) break;
#if IKPSO_COOP_TIMING
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
            if constexpr (PBG)
                swarm_step_pbg<Topo, MODE, TERMS, BLOCK>(cc, sh, s_pb, pbg, tid, x, pbf, coef, rng);
            else
                swarm_step<Topo, MODE, TERMS, BLOCK>(cc, sh, s_pb, tid, x, v, pbf, coef, rng);
            const bool act = cs.member * BLOCK + tid < P;
            const uint32_t key = act ? ordered_key(pbf) : 0xFFFFFFFFu;
#if IKPSO_COOP_TIMING
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#endif
            if constexpr (PBG)
                coop_exchange<Topo, BLOCK>(sh, cs, pbg, key, io.coop_error, io.coop_spin_limit, false);
            else
                coop_exchange<Topo, BLOCK>(sh, cs, s_pb, key, io.coop_error, io.coop_spin_limit, false);
#if IKPSO_COOP_TIMING
            const unsigned long long t2 = __builtin_amdgcn_s_memtime();
            t_step += t1 - t0;  // wave 0's own step
            t_bar += cs.t_mid - t1;  // the local argmin: waiting at its barrier for the other waves' steps
            t_exch += t2 - cs.t_mid;  // the cross-CU hand-off + the closing barrier
            ++n_it;
#endif
        }
#if IKPSO_COOP_TIMING
        if (tid == 0) {
            unsigned long long* tm = io.coop_timing + (size_t)blockIdx.x * 4;
            tm[0] += t_step;
            tm[1] += t_exch;
            tm[2] += n_it;
            tm[3] += t_bar;
        }
#endif

        compiler_fence();
        const int member = cs.member;
        const int64_t bb = cs.b;
        const int ii = member * BLOCK + tid;
        if (member == 0) {  // outputs (updateGlobalBestCoordsKernel) + fitness + residual
            store_angles<Topo>(cc, io.out_angles, bb, tid, tid < D ? sh.g[tid] : 0.0f);
            if (tid == 0 && io.out_fitness) io.out_fitness[bb] = key_to_float(cs.gkey);
            if (io.out_residual && tid < 64) {
                float g[D];
#pragma unroll
                for (int d = 0; d < D; ++d) g[d] = sh.g[d];
                const float r = residual<Topo, MODE, TERMS>(cc, g, sh.tgt, sh.dh);
                if (tid == 0) io.out_residual[bb] = r;
            }
        }
        if (ii < P) {
            store_rng(rng, io.rng + bb * P + ii);
            if (io.dump_particles) {  // reference particles layout [3][D][P] per swarm
                float* base = io.dump_particles + bb * (int64_t)3 * D * P;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    base[(int64_t)d * P + ii] = x[d];
                    if constexpr (PBG) {
                        base[(int64_t)(D + d) * P + ii] = s_pb[d * BLOCK + tid];
                        base[(int64_t)(2 * D + d) * P + ii] = pbg.template ld<BLOCK>(d);
                    } else {
                        base[(int64_t)(D + d) * P + ii] = v[d];
                        base[(int64_t)(2 * D + d) * P + ii] = s_pb[d * BLOCK + tid];
                    }
                }
            }
            if (io.dump_bests) io.dump_bests[bb * P + ii] = pbf;
        }
        __syncthreads();  // sh / s_pb are reused by the next swarm; every wave has read cs
        if (cs.abort) {     // a wait timed out: mark this and every later swarm of the group as failed
            if (member == 0)
                for (int64_t r = bb; r < io.num_swarms; r += io.coop_ng) {
                    if (tid < cc.dfree) io.out_angles[r * cc.dfree + tid] = __builtin_nanf("");
                    if (tid == 0 && io.out_fitness) io.out_fitness[r] = __builtin_nanf("");
                    if (tid == 0 && io.out_residual) io.out_residual[r] = __builtin_nanf("");
                }
            break;
        }
        if (tid == 0) cs.b = bb + io.coop_ng;
        __syncthreads();
    }
}

// Launch: grid = NG * G workgroups, at most one per CU.  Co-residency is
// checked here against the occupancy query (the check hipLaunchCooperativeKernel
// would make; a plain launch gives the same residency without the cooperative
// queue): an oversized grid is an error, never a hang.
template <class Topo, int MODE, int TERMS, int T>
inline hipError_t launch_coop_block(const ChainConsts<Topo::J>& cc, const SwarmIO& io, hipStream_t stream)
{
    const auto kernel = &k_swarm_coop<Topo, MODE, TERMS, T>;
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, T, 0);
    if (e != hipSuccess) return e;
    const int64_t grid = (int64_t)io.coop_ng * io.coop_g;
    if (per_cu < 1 || grid > (int64_t)cus) return hipErrorCooperativeLaunchTooLarge;
    hipLaunchKernelGGL(kernel, dim3((unsigned)grid), dim3(T), 0, stream, cc, io);
    return hipGetLastError();
}

template <class Topo, int MODE, int TERMS>
inline hipError_t launch_coop_kernel(const ChainConsts<Topo::J>& cc, const SwarmIO& io, hipStream_t stream)
{
    if constexpr (kCoopThreads<Topo::D>() != kCoopLatencyThreads) {
        if (io.coop_block == kCoopLatencyThreads)
            return launch_coop_block<Topo, MODE, TERMS, kCoopLatencyThreads>(cc, io, stream);
    }
    if (io.coop_block != kCoopThreads<Topo::D>()) return hipErrorInvalidValue;
    return launch_coop_block<Topo, MODE, TERMS, kCoopThreads<Topo::D>()>(cc, io, stream);
}

template <class Topo, int MODE>
inline hipError_t run_coop(const ChainHost& ch, const SwarmIO& io, hipStream_t stream)
{
    const ChainConsts<Topo::J> cc = make_consts<Topo::J>(ch);
    const int terms = term_set(ch);
    hipError_t err = hipSuccess;
    if (dh_terms<Topo>(terms, &err,
                       [&](auto t) { return launch_coop_kernel<Topo, MODE, decltype(t)::value>(cc, io, stream); }))
        return err;
    if constexpr (!Topo::kGeneric && !Topo::kDH && MODE == IKPSO_ARITH_FAST) {
        if (terms == kTermUniformBounds) return launch_coop_kernel<Topo, MODE, kTermUniformBounds>(cc, io, stream);
        if (terms == (kTermUniformBounds | kTermPenalty))
            return launch_coop_kernel<Topo, MODE, kTermUniformBounds | kTermPenalty>(cc, io, stream);
    }
    return with_runtime_terms<Topo>(
        ch, [&](auto t) { return launch_coop_kernel<Topo, MODE, decltype(t)::value>(cc, io, stream); });
}

}  // namespace ikpso
