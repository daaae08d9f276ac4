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
// slots hold zeros or the tags of earlier launches: a launch numbers its
// exchanges past them (io.coop_tag0; the host zeroes the slots when the
// numbering would wrap or the region was used for something else), so neither
// tag 0 nor a stale tag ever matches.  Workgroup b sits
// on XCD b % 8; the G chunks of a group share an XCD (speed only, never
// correctness) -- except a latency group wider than an XCD (the visualiser's
// N = 16384: 64 chunks), which takes linear membership and hands off across
// XCDs (coop_membership).  Waits are bounded: a timed-out wait sets io.coop_error and
// the kernel drains.
// Residency is checked at launch against the occupancy query.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
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
    unsigned long long t_ahead_sum;  // wave 0's publish + draws ahead, summed over the exchanges
    unsigned int n_imp, n_remote, n_polls;  // improving exchanges, ... won by another chunk, key polls
#endif
};

// Group membership of a cooperative workgroup: XCD-aware (workgroups b, b+8,
// b+16, ... share an XCD, so a group's chunks share an L2) or, for a latency
// group wider than an XCD, linear.
__device__ __forceinline__ void coop_membership(const SwarmIO& io, int* group, int* member)
{
    const int G = io.coop_g;
    if (io.coop_linear) {
        *group = blockIdx.x / G;
        *member = blockIdx.x % G;
    } else {
        const int xcd = blockIdx.x & 7, pos = blockIdx.x >> 3;
        *group = (pos / G) * 8 + xcd;
        *member = pos % G;
    }
}

// Exchange `e` of a group: publish this chunk's local argmin, wait for the G
// chunks, reduce; returns the group-wide minimum key of this exchange (uniform)
// and leaves the winner's local best in sh.g when it improves on `gkey` (or
// always when `force`).  Called by every wave; wave 0 does the global work.
// ahead(): gbest-independent work of the next iteration, done while the
// exchange is in flight (wave 0 between its publish and its poll, the other
// waves while wave 0 hands off) when do_ahead.
template <class Topo, int BLOCK, class AheadFn>
__device__ __forceinline__ void coop_exchange(SwarmShared<Topo>& sh, CoopShared<Topo::J>& cs, const float* s_pb,
                                              uint32_t local_key, int32_t* error, uint32_t spin_limit, bool force,
                                              bool do_ahead, AheadFn&& ahead)
{
    constexpr int D = Topo::D;
    constexpr int SLOT = kCoopSlot(D);
    static_assert(D + 1 <= 64, "wave 0 publishes the record in one store instruction");
    int lidx;
    const uint32_t lmin = swarm_argmin(sh, 0, local_key, &lidx);  // one workgroup barrier inside
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
        const float mine_d = lane >= 1 && lane <= D ? s_pb[(lane - 1) * BLOCK + lidx] : 0.0f;
        // Short chains (kPollFirst): the other chunks' key granules are requested BEFORE
        // this chunk's record is stored (its own key is known), so the first poll's
        // wait does not include the store's write-through (vmcnt counts stores).
        // Every lane loads -- lanes past G re-read chunk 0's key -- so no lane's branch
        // has to wait for the load before the store issues.  Config 2: 1.394 -> 1.342
        // ms; config 5 (D = 60): no gain (61.3 vs 61.5 ms), so not there
        // (profiles/r03m/variant_timings/var_*_pf.txt).
        constexpr bool kPollFirst = D <= 30;
        granule_t kraw = kPollFirst ? ld_granule(base + (size_t)(lane < G ? lane : 0) * SLOT) : tag;
        if (lane <= D) st_granule(base + (size_t)member * SLOT + lane, tag | (lane == 0 ? lmin : __float_as_uint(mine_d)));
        if (do_ahead) ahead();
#if IKPSO_COOP_TIMING
        cs.t_ahead_sum += __builtin_amdgcn_s_memtime() - cs.t_mid;
#endif
        // the G key granules, in chunk order (lanes 0..G-1; G <= 64)
        uint32_t n = 0;
        int timed_out = 0;
        granule_t kg;
        for (int first = 1;; first = 0) {
            if constexpr (kPollFirst) {
                if (!first) kraw = ld_granule(base + (size_t)(lane < G ? lane : 0) * SLOT);
                kg = lane == member ? (tag | lmin) : lane < G ? kraw : tag;
            } else {
                kg = lane < G ? ld_granule(base + (size_t)lane * SLOT) : tag;
            }
            if (__builtin_amdgcn_ballot_w64((kg >> 32) != (granule_t)(e + 1)) == 0) break;
            if (spin_limit == 0 || n++ >= spin_limit) {  // spin_limit 0 (IKPSO_COOP_SPIN_LIMIT=0): the give-up path
                timed_out = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
#if IKPSO_COOP_TIMING
        if (lane == 0) cs.n_polls += n + 1;
#endif
        const uint32_t k = lane < G ? (uint32_t)kg : 0xFFFFFFFFu;
        const uint32_t gmin = wave_min_u32(k);
        const int wj = wave_first_lane_eq(k, gmin);
        const uint32_t cur = cs.gkey;
        if (!timed_out && (force || gmin < cur)) {  // uniform within wave 0
#if IKPSO_COOP_TIMING
            if (lane == 0 && !force) {
                cs.n_imp += 1;
                cs.n_remote += wj != member;
            }
#endif
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
                // system scope: the flag may live in pinned host memory (the per-frame call)
                __hip_atomic_store(error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    } else if (do_ahead) {
        ahead();
    }
    __syncthreads();
}

// Dimensions of the next iteration's update drawn ahead during the exchange,
// in the throughput build of the FAST tip-backward (long-chain, 2-wave) step:
// wave 0 draws them between its publish and its poll, the other waves while
// wave 0 hands off, so the hand-off's wait carries work.  Config 5, 2048 swarms
// x 4096 x 100: 3 dimensions (node 1) 64.4 -> 63.3 ms; round 3 measured 6 and 9 no
// better than 3 (the extra live values spilled); with the velocities updated in
// their own registers (fma_inplace) the loop has room: 3 / 6 / 9 dimensions
// 58.36 / 58.22 / 58.08 ms (profiles/r04/variant_timings/var_c5b.txt).
#ifndef IKPSO_COOP_AHEAD_DIMS
#define IKPSO_COOP_AHEAD_DIMS 9
#endif
template <class Topo, int MODE, int TERMS, int BLOCK>
constexpr int kCoopAhead = (kTipBackward<Topo, MODE, TERMS> && Topo::D > 30) ? IKPSO_COOP_AHEAD_DIMS : 0;
// Waves per SIMD a cooperative build is compiled for: its own (BLOCK / 256)
// times the workgroups that share a CU (the latency variant: 1, alone on its
// CU).  The long chains' collider builds need more than 256 VGPRs: compiled for
// one workgroup per CU, and launch_coop_block fits the groups to that.
template <int D, int BLOCK, int TERMS>
constexpr int kCoopMinWaves = (BLOCK >= 256 ? BLOCK / 256 : 1) *
                              (BLOCK == kCoopThreads<D>() && !(TERMS & kTermColliders) ? kCoopBlocksPerCU<D>() : 1);
// Pricing builds of a third wave per SIMD for the long chains (variants only): the
// register budget of three workgroups per CU (168 VGPRs) while LDS still admits two --
// what the spills alone cost.
#ifndef IKPSO_EXPERIMENT_COOP_WAVES3
#define IKPSO_EXPERIMENT_COOP_WAVES3 0
#endif
template <int D, int BLOCK, int TERMS>
constexpr int kCoopBoundWaves =
    (IKPSO_EXPERIMENT_COOP_WAVES3 && D > 30 && BLOCK == kCoopThreads<D>() && !(TERMS & kTermColliders))
        ? 3 : kCoopMinWaves<D, BLOCK, TERMS>;

// BLOCK: kCoopThreads<D>() (throughput: fill each CU), or kCoopLatencyThreads
// for a few swarms (latency: one wave per SIMD on 4x more CUs).
template <class Topo, int MODE, int TERMS, int BLOCK>
__global__ void __launch_bounds__(BLOCK, (kCoopBoundWaves<Topo::D, BLOCK, TERMS>))
    k_swarm_coop(const ChainConsts<Topo::J> cc, const SwarmIO io)
{
    constexpr int J = Topo::J;
    constexpr int D = Topo::D;
    const int tid = threadIdx.x;
    const int P = io.P;

    // local bests [d][lane]; a build that owns its CU is padded to > 80 KiB so a
    // CU never holds two of its workgroups (the launch geometry assumes one)
    constexpr bool kOwnCU = kCoopMinWaves<D, BLOCK, TERMS> == (BLOCK >= 256 ? BLOCK / 256 : 1);
    constexpr int kPb = (!kOwnCU || D * BLOCK * 4 > 82 * 1024) ? D * BLOCK : 82 * 1024 / 4;
    __shared__ SwarmLds<Topo, kPb, CoopShared<J>> lds;
    SwarmShared<Topo>& sh = lds.sh;
    CoopShared<J>& cs = lds.extra;
    float* const s_pb = lds.pb;
    if (tid == 0) {
        const int G = io.coop_g;
        int group, member;
        coop_membership(io, &group, &member);
        cs.G = G;
        cs.member = member;
        cs.e = io.coop_tag0;
        cs.abort = 0;
        cs.b = group;
#if IKPSO_COOP_TIMING
        cs.n_imp = cs.n_remote = cs.n_polls = 0;
        cs.t_ahead_sum = 0;
#endif
        cs.slots = io.coop_slots + (size_t)group * 2 * G * kCoopSlot(D);
    }
    __syncthreads();
    const PsoCoef coef = pso_coef(cc);

    for (;;) {
        compiler_fence();
        const int64_t b = cs.b;
        if (b >= io.num_swarms) break;
        const int i = cs.member * BLOCK + tid;  // particle index within the swarm
        stage_swarm_inputs<Topo, TERMS>(cc, io.targets, io.start_pose, b, sh);
        // the add-for-shift issue form (t + t for t << 1) in the latency variant
        // (one wave per SIMD, room to spare) and in the long-chain build: 2 %
        // faster on config 5's two-chunks-per-CU kernel (profiles/r03f
        // variant_timings), where round 2's one-512-lane-chunk kernel had
        // measured it 5 % slower; the short chains' 1024-lane cooperative build keeps the shift
        using Rng = XorwowT<((kOwnCU && BLOCK == kCoopLatencyThreads) || D > 30) &&
                            std::is_same_v<RngFor<TERMS>, XorwowT<true>>>;
        Rng rng{0, 0, 0, 0, 0, 0};
        if (i < P) {
            if (io.rng_snap) io.rng_snap[b * P + i] = io.rng[b * P + i];  // the whole 48-byte state
            load_rng(rng, io.rng + b * P + i);
        }
        if (tid == 0) cs.gkey = 0xFFFFFFFFu;
        __syncthreads();

        // initParticlesKernel + initLocalBests (src/kernel.cu:191-266)
        float x[D], v[D];
        init_particle<Topo, TERMS, BLOCK>(cc, sh, s_pb, tid, x, v, rng);
        // the next iteration's first KA dimensions drawn ahead, inside the exchange
        constexpr int KA = kCoopAhead<Topo, MODE, TERMS, BLOCK>;
        float pa[KA > 0 ? KA : 1], pc[KA > 0 ? KA : 1];
        auto ahead = [&]() {
#pragma unroll
            for (int d = 0; d < KA; ++d) pso_draw_ahead(pa[d], pc[d], x[d], v[d], s_pb[d * BLOCK + tid], coef, rng);
        };
        float pbf = fitness<Topo, MODE, TERMS>(cc, x, sh.rest, sh.tgt, nullptr, sh.dh, sh.soft);
        // swarm argmin + unconditional first global-best copy (src/kernel.cu:297-304)
        const uint32_t key0 = i < P ? ordered_key(pbf) : 0xFFFFFFFFu;
        coop_exchange<Topo, BLOCK>(sh, cs, s_pb, key0, io.coop_error, io.coop_spin_limit, true, io.iterations > 0, ahead);

#if IKPSO_COOP_TIMING
        unsigned long long t_step = 0, t_bar = 0, t_exch = 0, n_it = 0;
#endif
        for (int it = 0; it < io.iterations; ++it) {
            compiler_fence();
            if (cs.abort) break;
#if IKPSO_COOP_TIMING
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
            if constexpr (KA > 0)
                swarm_step_tip<Topo, MODE, TERMS, BLOCK, KA, !kOwnCU>(cc, sh, s_pb, tid, x, v, pbf, coef, rng, pa,
                                                                     pc);  // inverted priority: two swarms per CU
            else
                swarm_step<Topo, MODE, TERMS, BLOCK>(cc, sh, s_pb, tid, x, v, pbf, coef, rng);
            const bool act = cs.member * BLOCK + tid < P;
            const uint32_t key = act ? ordered_key(pbf) : 0xFFFFFFFFu;
#if IKPSO_COOP_TIMING
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#endif
            coop_exchange<Topo, BLOCK>(sh, cs, s_pb, key, io.coop_error, io.coop_spin_limit, false,
                                       it + 1 < io.iterations, ahead);
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
            unsigned long long* tm = io.coop_timing + (size_t)blockIdx.x * 8;
            tm[0] += t_step;
            tm[1] += t_exch;
            tm[2] += n_it;
            tm[3] += t_bar;
            tm[4] += cs.n_imp;
            tm[5] += cs.n_remote;
            tm[6] += cs.n_polls;
            tm[7] += cs.t_ahead_sum;
            cs.n_imp = cs.n_remote = cs.n_polls = 0;
            cs.t_ahead_sum = 0;
        }
#endif

        compiler_fence();
        const int member = cs.member;
        const int64_t bb = cs.b;
        const int ii = member * BLOCK + tid;
        if (member == 0) {  // outputs (updateGlobalBestCoordsKernel) + fitness + residual
            store_angles<Topo, TERMS>(cc, io.out_angles, bb, tid, tid < D ? sh.g[tid] : 0.0f);
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
                    base[(int64_t)d * P + ii] = radians<TERMS>(x[d]);
                    base[(int64_t)(D + d) * P + ii] = radians<TERMS>(v[d]);
                    base[(int64_t)(2 * D + d) * P + ii] = radians<TERMS>(s_pb[d * BLOCK + tid]);
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

// The device's CU count and a kernel's resident workgroups per CU, queried once per
// (kernel, device) -- a latency-bound caller (the visualiser's per-frame call)
// launches thousands of times.
struct ResidencyCache {
    std::mutex mu;
    int dev = -1, cus = 0, per_cu = 0;
};
// `cache` is the launching function's own static: one per kernel instantiation.
template <class K>
inline hipError_t coop_residency(ResidencyCache& cache, K kernel, int threads, int* cus, int* per_cu)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(cache.mu);
    if (dev != cache.dev) {
        int n = 0, p = 0;
        e = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&p, kernel, threads, 0);
        if (e != hipSuccess) return e;
        cache.dev = dev, cache.cus = n, cache.per_cu = p;
    }
    *cus = cache.cus;
    *per_cu = cache.per_cu;
    return hipSuccess;
}

// Launch: grid = NG * G workgroups, at most kCoopBlocksPerCU per CU.  Co-residency is
// checked here against the occupancy query (the check hipLaunchCooperativeKernel
// would make; a plain launch gives the same residency without the cooperative
// queue): an oversized grid is an error, never a hang.
template <class Topo, int MODE, int TERMS, int T>
inline hipError_t launch_coop_block(const ChainConsts<Topo::J>& cc, const SwarmIO& io, hipStream_t stream)
{
    const auto kernel = &k_swarm_coop<Topo, MODE, TERMS, T>;
    static ResidencyCache cache;
    int cus = 0, per_cu = 0;
    const hipError_t e = coop_residency(cache, kernel, T, &cus, &per_cu);
    if (e != hipSuccess) return e;
    // The plan assumed kCoopBlocksPerCU workgroups per CU; a build whose registers
    // admit fewer (the long chains' collider builds exceed 256 VGPRs) runs fewer
    // concurrent groups -- the slots carved for the plan's NG cover them.
    const int want_per_cu = kCoopMinWaves<Topo::D, T, TERMS> / (T >= 256 ? T / 256 : 1);
    const int fit = per_cu < want_per_cu ? per_cu : want_per_cu;
    if (fit < 1) return hipErrorCooperativeLaunchTooLarge;
    SwarmIO run = io;
    const int ng_fit = io.coop_linear ? cus * fit / io.coop_g : (int)(((int64_t)cus * fit / io.coop_g) & ~int64_t(7));
    if (ng_fit < (io.coop_linear ? 1 : 8)) return hipErrorCooperativeLaunchTooLarge;
    if (run.coop_ng > ng_fit) run.coop_ng = ng_fit;
    const int64_t grid = (int64_t)run.coop_ng * run.coop_g;
    hipLaunchKernelGGL(kernel, dim3((unsigned)grid), dim3(T), 0, stream, cc, run);
    return hipGetLastError();
}

// ------------------------------------------------ latency variant, generator split
// A swarm spread thin (config 2: 1024 particles over 4 CUs, one wave per SIMD)
// is bound by ONE wave's instruction stream per iteration: a lone wave issues at
// most every 4 cycles (8 for the half-rate and transcendental forms), so the
// step takes ~5 900 cycles for 1 079 instructions (IKPSO_COOP_TIMING,
// profiles/r03f/variant_timings/var_r7_latency.txt) while three of a SIMD's
// four issue slots stay empty.  More than half of those instructions are the
// XORWOW generator, which depends on nothing but its own state.  Here each
// 256-particle chunk gets 512 lanes: waves 0-3 compute (update, FK, fitness,
// local bests, exchange) and waves 4-7 run the generators of the same 256
// particles one iteration ahead, writing each draw converted to float
// (v_cvt_f32_u32 of the XORWOW output, exactly what uniform()/scaled() start
// from) into an LDS block [quad][lane][4]; the compute lanes read four draws per
// ds_read_b128 and finish them with the one FMA of uniform()/scaled().  The draw
// order, the values and the final generator states are the unsplit kernel's,
// bit for bit, in both arithmetic modes.  Block m (0: the D init draws, m >= 1:
// the 3D draws of iteration m - 1) lives in buffer m & 1; the generator waves
// produce block m while iteration m - 2 runs -- quads [0, QA) beside the compute
// waves' step, the rest while wave 0 hands the chunk's minimum off -- so the two
// buffers alternate behind the exchange's barriers.  LDS: 2 x 64 KiB of draw
// blocks + 21 KiB of local bests at D = 21, so D <= 21; masked chains (their draw
// count is a runtime mask) and collider builds keep the unsplit latency kernel.
template <class Topo, int TERMS>
constexpr bool kSplitGen = IKPSO_SPLIT_GEN && Topo::D <= 21 && !kMasked<Topo, TERMS> && !(TERMS & kTermColliders);
template <int D>
constexpr int kSplitQuads = (3 * D + 3) / 4;  // float4 quads of the largest block (an iteration's 3D draws)
// quads of an iteration block the generator waves write beside the step (the rest during the hand-off)
template <int D>
constexpr int kSplitQA = IKPSO_SPLIT_QA < 0 ? kSplitQuads<D> / 2 : (IKPSO_SPLIT_QA < kSplitQuads<D> ? IKPSO_SPLIT_QA : kSplitQuads<D>);

// The compute lanes' draw source: the interface of XorwowT over one lane's
// column of an LDS block.  Fully unrolled callers make k a constant at every
// call site, so each quad is one ds_read_b128 at an immediate offset.
// PRE (iteration blocks): each draw already carries its PSO coefficient --
// c * uniform() as pso_update forms it -- so scaled() and the REFERENCE
// update's products take it as it is (kPrescaled); the init block holds
// (float)next() for uniform().
template <int BC, bool PRE>
struct LdsDraws {
    static constexpr bool kPrescaled = PRE;
    const float4* p;  // the lane's column: p[q * BC] holds draws 4q .. 4q + 3
    int k;
    float4 cur;
    __device__ __forceinline__ float raw()
    {
        if ((k & 3) == 0) cur = p[(k >> 2) * BC];
        const int c = k & 3;
        ++k;
        return c == 0 ? cur.x : c == 1 ? cur.y : c == 2 ? cur.z : cur.w;
    }
    __device__ __forceinline__ float uniform() { return __builtin_fmaf(raw(), 2.3283064e-10f, 1.16415322e-10f); }
    __device__ __forceinline__ float scaled(float q, float h)
    {
        if constexpr (PRE)
            return raw();
        else
            return __builtin_fmaf(raw(), q, h);
    }
};

// Generator lanes: quads [Q0, Q1) of a block of N draws into the lane's column.
// Init block (MODE < 0): (float)next().  Iteration blocks: draw j is r1, r2 or r3
// (j % 3) of its dimension, stored times its coefficient exactly as pso_update
// forms it -- FAST fma((float)next(), c * 2^-32, c * 2^-33) (scaled()), REFERENCE
// c * uniform() (the reference's first product, k.w * r1, ...).
template <int N, int Q0, int Q1, int BC, int MODE, class Rng>
__device__ __forceinline__ void gen_quads(Rng& rng, float4* col, const PsoCoef& k)
{
#pragma unroll
    for (int q = Q0; q < Q1; ++q) {
        float f[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int j = 4 * q + c;
            if (j >= N) {
                f[c] = 0.0f;
            } else if constexpr (MODE < 0) {
                f[c] = (float)rng.next();
            } else if constexpr (MODE == IKPSO_ARITH_FAST) {
                const float qq = j % 3 == 0 ? k.wq : j % 3 == 1 ? k.c1q : k.c2q;
                const float hh = j % 3 == 0 ? k.wh : j % 3 == 1 ? k.c1h : k.c2h;
                f[c] = rng.scaled(qq, hh);
            } else {
                const float cc = j % 3 == 0 ? k.w : j % 3 == 1 ? k.c1 : k.c2;
                const float r = rng.uniform();
                {
#pragma clang fp contract(off)
                    f[c] = cc * r;
                }
            }
        }
        col[q * BC] = make_float4(f[0], f[1], f[2], f[3]);
    }
}

template <class Topo, int BC>
struct SplitLds {
    static constexpr int D = Topo::D, NQ = kSplitQuads<Topo::D>;
    SwarmShared<Topo> sh;
    CoopShared<Topo::J> cs;
    float pb[D * BC];            // local bests [d][lane]
    float4 draws[2][NQ * BC];    // draw blocks [buffer][quad][lane]
    // more than half of a CU's LDS: one workgroup per CU (the launch plan's geometry)
    char pad[(int)sizeof(SwarmShared<Topo>) + D * BC * 4 + 2 * NQ * BC * 16 > 82 * 1024
                 ? 1
                 : 82 * 1024 - (int)sizeof(SwarmShared<Topo>) - D * BC * 4 - 2 * NQ * BC * 16];
};

template <class Topo, int MODE, int TERMS>
__global__ void __launch_bounds__(2 * kCoopLatencyThreads) k_swarm_coop_split(const ChainConsts<Topo::J> cc,
                                                                               const SwarmIO io)
{
    constexpr int D = Topo::D;
    constexpr int BC = kCoopLatencyThreads;  // particles per chunk = compute lanes = generator lanes
    constexpr int NQ = kSplitQuads<D>, QA = kSplitQA<D>;
    constexpr int NQI = (D + 3) / 4;  // quads of the init block
    __shared__ SplitLds<Topo, BC> lds;
    SwarmShared<Topo>& sh = lds.sh;
    CoopShared<Topo::J>& cs = lds.cs;
    float* const s_pb = lds.pb;
    const int tid = threadIdx.x;
    const bool gen = wave_id() >= BC / 64;  // uniform per wave
    const int lc = gen ? tid - BC : tid;    // the particle (within the chunk) this lane serves
    const int P = io.P;
    if (tid == 0) {
        const int G = io.coop_g;
        int group, member;
        coop_membership(io, &group, &member);
        cs.G = G;
        cs.member = member;
        cs.e = io.coop_tag0;
        cs.abort = 0;
        cs.b = group;
#if IKPSO_COOP_TIMING
        cs.n_imp = cs.n_remote = cs.n_polls = 0;
        cs.t_ahead_sum = 0;
#endif
        cs.slots = io.coop_slots + (size_t)group * 2 * G * kCoopSlot(D);
    }
    __syncthreads();
    const PsoCoef coef = pso_coef(cc);

    for (;;) {
        compiler_fence();
        const int64_t b = cs.b;
        if (b >= io.num_swarms) break;
        const int i = cs.member * BC + lc;
        stage_swarm_inputs<Topo, TERMS>(cc, io.targets, io.start_pose, b, sh);
        using Rng = XorwowT<std::is_same_v<RngFor<TERMS>, XorwowT<true>>>;  // add-for-shift: see k_swarm_coop
        Rng rng{0, 0, 0, 0, 0, 0};
        const int I = io.iterations;
        if (gen) {
            if (i < P) {
                if (io.rng_snap) io.rng_snap[b * P + i] = io.rng[b * P + i];
                load_rng(rng, io.rng + b * P + i);
            }
            gen_quads<D, 0, NQI, BC, -1>(rng, lds.draws[0] + lc, coef);  // block 0: initParticlesKernel's draws
        }
        if (tid == 0) cs.gkey = 0xFFFFFFFFu;
        __syncthreads();

        float x[D], v[D], pbf = 0.0f;
#pragma unroll
        for (int d = 0; d < D; ++d) x[d] = v[d] = 0.0f;
        if (!gen) {
            LdsDraws<BC, false> rd{lds.draws[0] + lc, 0, {}};
            init_particle<Topo, TERMS, BC>(cc, sh, s_pb, lc, x, v, rd);
            pbf = fitness<Topo, MODE, TERMS>(cc, x, sh.rest, sh.tgt, nullptr, sh.dh, sh.soft);
        } else if (I > 0) {
            gen_quads<3 * D, 0, QA, BC, MODE>(rng, lds.draws[1] + lc, coef);
        }
        // the rest of block m + 2 (into buffer m & 1) while wave 0 hands off
        int nb = 1;  // the block the generator waves are producing
        auto ahead = [&]() {
            if (gen) gen_quads<3 * D, QA, NQ, BC, MODE>(rng, lds.draws[nb & 1] + lc, coef);
        };
        const uint32_t key0 = !gen && i < P ? ordered_key(pbf) : 0xFFFFFFFFu;
        coop_exchange<Topo, BC>(sh, cs, s_pb, key0, io.coop_error, io.coop_spin_limit, true, I > 0, ahead);

#if IKPSO_COOP_TIMING
        unsigned long long t_step = 0, t_bar = 0, t_exch = 0, n_it = 0;
#endif
        for (int it = 0; it < I; ++it) {
            compiler_fence();
            if (cs.abort) break;
#if IKPSO_COOP_TIMING
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
            nb = it + 2;
            if (!gen) {
                LdsDraws<BC, true> rd{lds.draws[(it + 1) & 1] + lc, 0, {}};
                swarm_step<Topo, MODE, TERMS, BC>(cc, sh, s_pb, lc, x, v, pbf, coef, rd);
            } else if (nb <= I) {
                gen_quads<3 * D, 0, QA, BC, MODE>(rng, lds.draws[nb & 1] + lc, coef);
            }
            const uint32_t key = !gen && i < P ? ordered_key(pbf) : 0xFFFFFFFFu;
#if IKPSO_COOP_TIMING
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#endif
            coop_exchange<Topo, BC>(sh, cs, s_pb, key, io.coop_error, io.coop_spin_limit, false, nb <= I, ahead);
#if IKPSO_COOP_TIMING
            const unsigned long long t2 = __builtin_amdgcn_s_memtime();
            t_step += t1 - t0;
            t_bar += cs.t_mid - t1;
            t_exch += t2 - cs.t_mid;
            ++n_it;
#endif
        }
#if IKPSO_COOP_TIMING
        if (tid == 0) {
            unsigned long long* tm = io.coop_timing + (size_t)blockIdx.x * 8;
            tm[0] += t_step;
            tm[1] += t_exch;
            tm[2] += n_it;
            tm[3] += t_bar;
            tm[4] += cs.n_imp;
            tm[5] += cs.n_remote;
            tm[6] += cs.n_polls;
            tm[7] += cs.t_ahead_sum;
            cs.n_imp = cs.n_remote = cs.n_polls = 0;
            cs.t_ahead_sum = 0;
        }
#endif

        compiler_fence();
        const int member = cs.member;
        const int64_t bb = cs.b;
        const int ii = member * BC + lc;
        if (!gen && member == 0) {  // outputs (updateGlobalBestCoordsKernel) + fitness + residual
            store_angles<Topo, TERMS>(cc, io.out_angles, bb, tid, tid < D ? sh.g[tid] : 0.0f);
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
            if (gen) {
                store_rng(rng, io.rng + bb * P + ii);
            } else {
                if (io.dump_particles) {  // reference particles layout [3][D][P] per swarm
                    float* base = io.dump_particles + bb * (int64_t)3 * D * P;
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        base[(int64_t)d * P + ii] = radians<TERMS>(x[d]);
                        base[(int64_t)(D + d) * P + ii] = radians<TERMS>(v[d]);
                        base[(int64_t)(2 * D + d) * P + ii] = radians<TERMS>(s_pb[d * BC + lc]);
                    }
                }
                if (io.dump_bests) io.dump_bests[bb * P + ii] = pbf;
            }
        }
        __syncthreads();  // sh / s_pb / the draw blocks are reused by the next swarm; every wave has read cs
        if (cs.abort) {
            if (member == 0 && !gen)
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

// One workgroup of 2 x kCoopLatencyThreads lanes per CU (the latency plan's geometry).
template <class Topo, int MODE, int TERMS>
inline hipError_t launch_coop_split(const ChainConsts<Topo::J>& cc, const SwarmIO& io, hipStream_t stream)
{
    const auto kernel = &k_swarm_coop_split<Topo, MODE, TERMS>;
    constexpr int T = 2 * kCoopLatencyThreads;
    static ResidencyCache cache;
    int cus = 0, per_cu = 0;
    const hipError_t e = coop_residency(cache, kernel, T, &cus, &per_cu);
    if (e != hipSuccess) return e;
    if (per_cu < 1) return hipErrorCooperativeLaunchTooLarge;
    SwarmIO run = io;
    const int ng_fit = io.coop_linear ? cus / io.coop_g : (int)(((int64_t)cus / io.coop_g) & ~int64_t(7));
    if (ng_fit < (io.coop_linear ? 1 : 8)) return hipErrorCooperativeLaunchTooLarge;
    if (run.coop_ng > ng_fit) run.coop_ng = ng_fit;
    const int64_t grid = (int64_t)run.coop_ng * run.coop_g;
    hipLaunchKernelGGL(kernel, dim3((unsigned)grid), dim3(T), 0, stream, cc, run);
    return hipGetLastError();
}

template <class Topo, int MODE, int TERMS>
inline hipError_t launch_coop_kernel(const ChainConsts<Topo::J>& cc, const SwarmIO& io, hipStream_t stream)
{
    if constexpr (kCoopThreads<Topo::D>() != kCoopLatencyThreads) {
        if (io.coop_block == kCoopLatencyThreads) {
            if constexpr (kSplitGen<Topo, TERMS>)
                return launch_coop_split<Topo, MODE, TERMS>(cc, io, stream);
            else
                return launch_coop_block<Topo, MODE, TERMS, kCoopLatencyThreads>(cc, io, stream);
        }
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
    // angles in revolutions in the specialised FAST and folded-chain builds (kTermRev)
    if (dh_terms<Topo>(terms, &err, [&](auto t) {
            return launch_coop_kernel<Topo, MODE, decltype(t)::value | kTermRev>(cc, io, stream);
        }))
        return err;
    if constexpr (!Topo::kGeneric && !Topo::kDH && MODE == IKPSO_ARITH_FAST) {
        if constexpr (std::is_same_v<Topo, TopoRef7>) {  // the reference scene's [0, 2pi] limits
            if (terms == kTermUniformBounds && ch.unit_rev_bounds)
                return launch_coop_kernel<Topo, MODE, kTermUniformBounds | kFastRev | kFastUnitBounds>(cc, io, stream);
        }
        if (terms == kTermUniformBounds)
            return launch_coop_kernel<Topo, MODE, kTermUniformBounds | kFastRev>(cc, io, stream);
        if constexpr (std::is_same_v<Topo, TopoSerialTip<20>>) {  // BASELINE config 5's symmetric soft limits
            if (terms == (kTermUniformBounds | kTermPenalty) && ch.sym_penalty)
                return launch_coop_kernel<Topo, MODE, kTermUniformBounds | kTermPenalty | kFastRev | kFastSymPenalty>(
                    cc, io, stream);
        }
        if (terms == (kTermUniformBounds | kTermPenalty))
            return launch_coop_kernel<Topo, MODE, kTermUniformBounds | kTermPenalty | kFastRev>(cc, io, stream);
    }
    return with_runtime_terms<Topo>(
        ch, [&](auto t) { return launch_coop_kernel<Topo, MODE, decltype(t)::value>(cc, io, stream); });
}

}  // namespace ikpso
