// ikpso_stream.h -- streaming variant of the swarm solve for swarms larger
// than one workgroup (the visualiser's default N = 16384, src/Main.cpp:17) and
// for long chains (BASELINE config 5: D = 60, P = 4096).
//
// Particle state lives in HBM in the reference's own SoA layout (per swarm
// [3][D][P]: position | velocity | local best, src/kernel.cu:17-29); one
// launch per PSO iteration covers every 256-particle chunk of every swarm, one
// lane per particle, coalesced [d][particle] loads/stores.  The swarm argmin
// (thrust::min_element, src/kernel.cu:297,315) is split across launches: each
// workgroup publishes its chunk minimum (key, index, the winner's pbest) to
// slot t&1, and every workgroup of the NEXT launch reduces those partials and
// applies the `globalMin > currentGlobalMin` update (src/kernel.cu:318)
// redundantly -- the kernel boundary is the only cross-workgroup ordering.
#pragma once

#include <hip/hip_runtime.h>

#include "ikpso_device.h"
#include "ikpso_kernels.h"
#include "ikpso_swarm.h"

namespace ikpso {

// Nodes of x / v / local best loaded ahead of their use in k_stream_step.
constexpr int kStreamAhead = 2;

// Resolve the swarm's global best as of the end of launch t-1: reduce the C
// chunk partials of slot (t-1)&1, compare with the global best of slot
// (t-1)&1, stage the resulting vector in sh.g.  Uniform across the workgroup.
// Workgroup 0 of each swarm publishes the result to slot t&1.
template <class Topo>
__device__ __forceinline__ uint32_t stream_resolve_gbest(const StreamIO& io, int64_t b, int c, SwarmShared<Topo>& sh)
{
    constexpr int D = Topo::D;
    const int lane = threadIdx.x & 63;
    const int prev = (io.t - 1) & 1, cur = io.t & 1;
    const int64_t B = io.num_swarms;
    const uint32_t* pk = io.pkey + ((int64_t)prev * B + b) * io.C;
    const int32_t* pi = io.pidx + ((int64_t)prev * B + b) * io.C;
    uint32_t best = 0xFFFFFFFFu;
    int best_chunk = 0;
    for (int base = 0; base < io.C; base += 64) {  // chunks in order: ties keep the lowest chunk
        const uint32_t k = base + lane < io.C ? pk[base + lane] : 0xFFFFFFFFu;
        const uint32_t m = wave_min_u32(k);
        if (m < best) {
            best = m;
            best_chunk = base + wave_first_lane_eq(k, m);
        }
    }
    const uint32_t gprev = io.gkey[(int64_t)prev * B + b];
    const bool improved = best < gprev;
    const float* src = improved ? io.pvec + (((int64_t)prev * B + b) * io.C + best_chunk) * D
                                : io.gvec + ((int64_t)prev * B + b) * D;
    for (int d = threadIdx.x; d < D; d += blockDim.x) sh.g[d] = src[d];
    if (c == 0) {
        if (threadIdx.x == 0) {
            io.gkey[(int64_t)cur * B + b] = improved ? best : gprev;
            io.gidx[(int64_t)cur * B + b] = improved ? pi[best_chunk] : io.gidx[(int64_t)prev * B + b];
        }
        for (int d = threadIdx.x; d < D; d += blockDim.x) io.gvec[((int64_t)cur * B + b) * D + d] = src[d];
    }
    return improved ? best : gprev;
}

// Chunk argmin of the local-best keys -> partial slot t&1; the winner lane
// publishes its pbest vector (its own stores of this launch, read back).
template <class Topo>
__device__ __forceinline__ void stream_publish_chunk(const StreamIO& io, int64_t b, int c, SwarmShared<Topo>& sh,
                                                     uint32_t key, const Planes& pl)
{
    constexpr int D = Topo::D;
    int widx;
    const uint32_t m = swarm_argmin(sh, 0, key, &widx);
    const int cur = io.t & 1;
    const int64_t slot = ((int64_t)cur * io.num_swarms + b) * io.C + c;
    if (threadIdx.x == 0) {
        io.pkey[slot] = m;
        io.pidx[slot] = c * kStreamChunk + widx;
    }
    if (threadIdx.x == widx) {
        float* dst = io.pvec + slot * D;
#pragma unroll
        for (int d = 0; d < D; ++d) dst[d] = pl.ld(2, d);
    }
}

template <class Topo, int MODE, int TERMS>
__global__ void __launch_bounds__(kStreamChunk) k_stream_init(const ChainConsts<Topo::J> cc, const StreamIO io)
{
    constexpr int D = Topo::D;
    const int64_t b = blockIdx.x / io.C;
    const int c = blockIdx.x % io.C;
    const int i = c * kStreamChunk + threadIdx.x;
    const bool active = i < io.P;
    const int64_t P = io.P;
    __shared__ SwarmShared<Topo> sh;
    stage_swarm_inputs<Topo>(cc, io.targets, io.start_pose, b, sh);
    __syncthreads();

    const Planes pl(io.state + b * 3 * D * P, D, (int)P, i);
    float x[D];
    float pbf = 0.0f;
    if (active) {
        // initParticlesKernel (src/kernel.cu:223-266) + initLocalBests (:191-200)
        RngFor<TERMS> rng;
        load_rng(rng, io.rng_aos + b * P + i);
#pragma unroll
        for (int d = 0; d < D; ++d) {
            x[d] = sh.rest[d];
            pl.st(0, d, x[d]);
            if (kMasked<Topo, TERMS> && !dim_free(cc, d))  // locked: no draw
                pl.st(1, d, 0.0f);
            else
                pl.st(1, d, __builtin_fmaf(rng.uniform(), 2.0f, -1.0f));
            pl.st(2, d, x[d]);
        }
        pbf = fitness<Topo, MODE, TERMS>(cc, x, sh.rest, sh.tgt, nullptr, sh.dh, sh.soft);
        io.pbf[b * P + i] = pbf;
        const int64_t n = io.num_swarms * P, k = b * P + i;
        io.rng[0 * n + k] = rng.d;
        io.rng[1 * n + k] = rng.v0;
        io.rng[2 * n + k] = rng.v1;
        io.rng[3 * n + k] = rng.v2;
        io.rng[4 * n + k] = rng.v3;
        io.rng[5 * n + k] = rng.v4;
    }
    stream_publish_chunk<Topo>(io, b, c, sh, active ? ordered_key(pbf) : 0xFFFFFFFFu, pl);
    if (c == 0 && threadIdx.x == 0) io.gkey[(int64_t)(io.t & 1) * io.num_swarms + b] = 0xFFFFFFFFu;
}

template <class Topo, int MODE, int TERMS>
__global__ void __launch_bounds__(kStreamChunk) k_stream_step(const ChainConsts<Topo::J> cc, const StreamIO io)
{
    constexpr int J = Topo::J, A = Topo::A;
    constexpr int D = Topo::D;
    const int64_t b = blockIdx.x / io.C;
    const int c = blockIdx.x % io.C;
    const int i = c * kStreamChunk + threadIdx.x;
    const bool active = i < io.P;
    const int64_t P = io.P;
    __shared__ SwarmShared<Topo> sh;
    stage_swarm_inputs<Topo>(cc, io.targets, io.start_pose, b, sh);
    stream_resolve_gbest<Topo>(io, b, c, sh);
    __syncthreads();

    const Planes pl(io.state + b * 3 * D * P, D, (int)P, i);
    float pbf = 0.0f;
    if (active) {
        const int64_t n = io.num_swarms * P, k = b * P + i;
        RngFor<TERMS> rng;
        rng.d = io.rng[0 * n + k];
        rng.v0 = io.rng[1 * n + k];
        rng.v1 = io.rng[2 * n + k];
        rng.v2 = io.rng[3 * n + k];
        rng.v3 = io.rng[4 * n + k];
        rng.v4 = io.rng[5 * n + k];
        pbf = io.pbf[b * P + i];
        // One node at a time: update its three angles (simulateParticlesKernel,
        // src/kernel.cu:153-189: draws r1, r2, r3 per dimension in dimension
        // order, then the clamp), store them, and fold the node into the
        // fitness (calculateDistance, src/kernel.cu:64-151).  A node's FK needs
        // only its own and its ancestors' angles, so this is the reference's
        // update-all-then-evaluate with the same values and accumulation order,
        // while only a handful of angles are live at a time.
        const PsoCoef coef = pso_coef(cc);
        // kTipBackward builds (serial chains with only the tip's position in the
        // fitness, and the folded chain): every node updated first, then the tip
        // evaluated from the tip back -- the form the resident and cooperative
        // kernels use (swarm_step_tip), so a streaming solve (or a cooperative
        // solve's fallback) rounds like them
        constexpr bool TIP = kTipBackward<Topo, MODE, TERMS>;
        CandBuf<Topo, TERMS> cb;
        FitnessFor<Topo, MODE, TERMS> acc(cc, sh.dh, sh.soft, cb.v);
        TipAccFor<Topo, MODE, TERMS> tb(sh.dh, sh.soft);
        float xs[TIP ? D : 1];
        // Loads are software-pipelined AHEAD nodes ahead (a ring of AHEAD+1
        // node slots in registers, indices resolved at compile time) and every
        // node ends in a scheduling barrier: left alone, the compiler hoists
        // all 9J loads to the top (256 VGPRs, one wave per SIMD,
        // latency-bound); one node ahead leaves HBM latency exposed.
        constexpr int AHEAD = (kStreamAhead < J) ? kStreamAhead : J;
        float ring[AHEAD + 1][3 * A];
#pragma unroll
        for (int s = 0; s < AHEAD; ++s)
#pragma unroll
            for (int ax = 0; ax < A; ++ax) {
                ring[s][ax] = pl.ld(0, A * s + ax);
                ring[s][A + ax] = pl.ld(1, A * s + ax);
                ring[s][2 * A + ax] = pl.ld(2, A * s + ax);
            }
#pragma unroll
        for (int kn = 1; kn <= J; ++kn) {
            float cx[A], cv[A], cpb[A];
            const int cs = (kn - 1) % (AHEAD + 1);
#pragma unroll
            for (int ax = 0; ax < A; ++ax) {
                cx[ax] = ring[cs][ax];
                cv[ax] = ring[cs][A + ax];
                cpb[ax] = ring[cs][2 * A + ax];
            }
            if (kn - 1 + AHEAD < J) {  // node kn + AHEAD (0-based kn - 1 + AHEAD)
                const int nn = kn - 1 + AHEAD, ns = nn % (AHEAD + 1);
#pragma unroll
                for (int ax = 0; ax < A; ++ax) {
                    ring[ns][ax] = pl.ld(0, A * nn + ax);
                    ring[ns][A + ax] = pl.ld(1, A * nn + ax);
                    ring[ns][2 * A + ax] = pl.ld(2, A * nn + ax);
                }
            }
#pragma unroll
            for (int ax = 0; ax < A; ++ax) {
                const int d = A * (kn - 1) + ax;
                if (kMasked<Topo, TERMS> && !dim_free(cc, d)) continue;  // locked: stays at rest
                pso_update<MODE>(cx[ax], cv[ax], cpb[ax], sh.g[d], coef, rng);
                pl.st(1, d, cv[ax]);
                if constexpr (TERMS & kTermUniformBounds)
                    cx[ax] = clamp_mode<MODE>(cx[ax], cc.lo[0], cc.hi[0]);
                else
                    cx[ax] = clamp_mode<MODE>(cx[ax], sh.lo[d], sh.hi[d]);
                pl.st(0, d, cx[ax]);
            }
            if constexpr (TIP) {
#pragma unroll
                for (int ax = 0; ax < A; ++ax) xs[A * (kn - 1) + ax] = cx[ax];
                tb.angles(kn, cx, sh.rest + A * (kn - 1));
            } else {
                acc.node(cc, kn, cx, sh.rest + A * (kn - 1), sh.tgt + 3 * (kn - 1), nullptr);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        float f;
        if constexpr (TIP) {
#pragma unroll
            for (int kn = J; kn >= 1; --kn) tb.back(cc, kn, node_trig<decltype(tb)::HW, A>(xs + A * (kn - 1)));
            f = tb.finish(cc, sh.tgt + 3 * (J - 1));
        } else {
            f = acc.finish_for_update(cc, pbf);
        }
        // updateLocalBests (src/kernel.cu:202-221)
        // Whole-line stores only: a store covering part of a 128-B line makes
        // the memory side fetch the line first.  A wave with no improving lane
        // writes nothing; otherwise every lane rewrites its local best (its new
        // position, or the old value read back -- an L2 hit, read by the update
        // above).
        const bool imp = f < pbf;
        pbf = imp ? f : pbf;
        if (__builtin_amdgcn_ballot_w64(imp)) {
            io.pbf[b * P + i] = pbf;
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const float xn = pl.ld(0, d), po = pl.ld(2, d);
                pl.st(2, d, imp ? xn : po);
            }
        }
        io.rng[0 * n + k] = rng.d;
        io.rng[1 * n + k] = rng.v0;
        io.rng[2 * n + k] = rng.v1;
        io.rng[3 * n + k] = rng.v2;
        io.rng[4 * n + k] = rng.v3;
        io.rng[5 * n + k] = rng.v4;
    }
    stream_publish_chunk<Topo>(io, b, c, sh, active ? ordered_key(pbf) : 0xFFFFFFFFu, pl);
}

template <class Topo, int MODE, int TERMS>
__global__ void __launch_bounds__(kStreamChunk) k_stream_finalize(const ChainConsts<Topo::J> cc, const StreamIO io)
{
    constexpr int D = Topo::D;
    const int64_t b = blockIdx.x / io.C;
    const int c = blockIdx.x % io.C;
    const int i = c * kStreamChunk + threadIdx.x;
    const int64_t P = io.P;
    __shared__ SwarmShared<Topo> sh;
    stage_swarm_inputs<Topo>(cc, io.targets, io.start_pose, b, sh);
    const uint32_t gkey = stream_resolve_gbest<Topo>(io, b, c, sh);
    __syncthreads();
    if (c == 0) {
        // Coordinates result (updateGlobalBestCoordsKernel) + fitness + residual
        for (int d = threadIdx.x; d < D; d += blockDim.x) store_angles<Topo>(cc, io.out_angles, b, d, sh.g[d]);
        if (threadIdx.x == 0 && io.out_fitness) io.out_fitness[b] = key_to_float(gkey);
        if (io.out_residual && threadIdx.x < 64) {
            float g[D];
#pragma unroll
            for (int d = 0; d < D; ++d) g[d] = sh.g[d];
            const float r = residual<Topo, MODE, TERMS>(cc, g, sh.tgt, sh.dh);
            if (threadIdx.x == 0) io.out_residual[b] = r;
        }
    }
    if (i < io.P) {  // generator states back to the caller's / solver's layout
        const int64_t n = io.num_swarms * P, k = b * P + i;
        Xorwow rng;
        rng.d = io.rng[0 * n + k];
        rng.v0 = io.rng[1 * n + k];
        rng.v1 = io.rng[2 * n + k];
        rng.v2 = io.rng[3 * n + k];
        rng.v3 = io.rng[4 * n + k];
        rng.v4 = io.rng[5 * n + k];
        store_rng(rng, io.rng_aos + k);
    }
}

template <class Topo, int MODE, int TERMS>
inline hipError_t run_stream(const ChainHost& ch, StreamIO io, int iterations, hipStream_t stream)
{
    const ChainConsts<Topo::J> cc = make_consts<Topo::J>(ch);
    const dim3 grid((unsigned)(io.num_swarms * io.C)), threads(kStreamChunk);
    io.t = 0;
    hipLaunchKernelGGL((k_stream_init<Topo, MODE, TERMS>), grid, threads, 0, stream, cc, io);
    for (int t = 1; t <= iterations; ++t) {
        io.t = t;
        hipLaunchKernelGGL((k_stream_step<Topo, MODE, TERMS>), grid, threads, 0, stream, cc, io);
    }
    io.t = iterations + 1;
    hipLaunchKernelGGL((k_stream_finalize<Topo, MODE, TERMS>), grid, threads, 0, stream, cc, io);
    return hipGetLastError();
}

template <class Topo, int MODE>
inline hipError_t run_stream_terms(const ChainHost& ch, const StreamIO& io, int iterations, hipStream_t stream)
{
    // Same term specialisation as run_resident.
    const int terms = term_set(ch);
    hipError_t err = hipSuccess;
    if (dh_terms<Topo>(terms, &err,
                       [&](auto t) { return run_stream<Topo, MODE, decltype(t)::value>(ch, io, iterations, stream); }))
        return err;
    if constexpr (!Topo::kGeneric && !Topo::kDH && MODE == IKPSO_ARITH_FAST) {
        if (terms == kTermUniformBounds) return run_stream<Topo, MODE, kTermUniformBounds>(ch, io, iterations, stream);
        if (terms == (kTermUniformBounds | kTermPenalty))
            return run_stream<Topo, MODE, kTermUniformBounds | kTermPenalty>(ch, io, iterations, stream);
    }
    (void)terms;
    return with_runtime_terms<Topo>(
        ch, [&](auto t) { return run_stream<Topo, MODE, decltype(t)::value>(ch, io, iterations, stream); });
}

}  // namespace ikpso
