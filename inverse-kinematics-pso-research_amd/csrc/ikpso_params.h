// ikpso_params.h -- kernel parameter blocks shared by host and device code.
#pragma once

#include <stdint.h>

#include "ikpso.h"

namespace ikpso {

constexpr int kMaxJoints = 32;

// Per-chain constants, passed by value so they land in the kernarg segment and
// are read with scalar loads (the chain is identical for every particle and
// every swarm, so it belongs in SGPRs, not in VGPRs or LDS).  Index k = node
// index (1..J); per-angle arrays are indexed d = 3*(k-1)+axis.
template <int J>
struct ChainConsts {
    float len[J + 1];
    float eff_w[J + 1];
    int32_t eff_slot[J + 1];  // effector ordinal among effectors, -1 otherwise
    int32_t parent[J + 1];    // used by the generic-topology kernels only
    float lo[3 * J], hi[3 * J];
    float rest[3 * J];        // default warm start / angle-term reference
    float tgt0[3 * J];        // chain's own effector targets, per node (k-1)
    float m0[12];             // origin world transform, rows 0..2 of the 4x4
    // Rarely used terms live in device memory, not in the kernarg segment (the
    // compiler hoists every kernarg load out of the PSO loop into SGPRs):
    // aux = [posref 4J | soft_lo 3J | soft_hi 3J].
    const float* aux;
    float w, c1, c2;          // inertia, local, global
    float aw_j, dw_j, lim_w;  // angleWeight/J, distanceWeight/J, limit weight
    int32_t use_posref, use_penalty;
    int32_t num_eff;
};

// Per-launch buffers.
struct SwarmIO {
    const float* targets;     // [B][E][3] or null (chain targets for every swarm)
    const float* start_pose;  // [B][D] or null
    ikpso_rng_state* rng;     // [B][P]
    float* out_angles;        // [B][D]
    float* out_fitness;       // [B] or null
    float* out_residual;      // [B] or null
    float* dump_particles;    // [B][3][D][P] or null (reference particles layout)
    float* dump_bests;        // [B][P] or null
    int32_t P;
    int32_t iterations;
    int64_t num_swarms;
};

// Streaming (state-in-HBM) kernels: per-swarm global-best state, double
// buffered by iteration parity.
struct GBest {
    uint32_t key;  // ordered fp32 key of the global-best fitness
    int32_t idx;   // particle index of the global best
};

}  // namespace ikpso
