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
    // The link lengths the FAST kernels on the transcendental unit's sin/cos use:
    // len[k] * (1 + 2 depth(k) eps), rounded once from fp64 (make_consts).  See
    // kHwTrigAmplitudeBias (ikpso_kernels.h) and link_len (ikpso_device.h).
    float len_hw[J + 1];
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
    float wq, c1q, c2q;       // the same times 2^-32 (exact): FAST mode folds
    float wh, c1h, c2h;       // the uniform's affine map, times 2^-33 (exact)
    float aw_j, dw_j, lim_w;  // angleWeight/J, distanceWeight/J, limit weight
    // kTermRev builds (angles in revolutions): the weights times (2 pi)^2 and the
    // uniform clamp bounds over 2 pi
    float aw_rev, lim_rev, rlo, rhi;
    int32_t use_posref, use_penalty;
    int32_t num_eff;
    int32_t num_coll;         // colliders (kTermColliders kernels only)
    const struct CollRec* coll;  // [num_coll] device records, inside the aux buffer
    const float* coll_lim;    // [J][num_coll] near_collider's squared limits, inside the aux buffer
    const float* coll_box;    // [num_coll][16] the colliders as oriented boxes (FAST separating-axis test,
                              // kFastSat): axes (3 columns), half extents, centre; inside the aux buffer
    unsigned long long* coll_stats;  // IKPSO_COLLIDE_STATS builds: [kCsCount] counters (else null)
    // Joint-axis mask (extension): bit d set when kernel
    // dimension d is a PSO dimension; dfree = popcount.  The kernels of the
    // Euler topologies run over all 3J Euler angles and honour the mask in their
    // runtime-term builds (locked angles stay at rest: no draws, no update, no
    // clamp); the API's angle vectors carry the dfree free dimensions only.
    uint64_t free_mask;
    int32_t dfree;
    // Folded serial chain (TopoDH): aux + dh_off holds, per joint j = 1..J, the
    // constant rotation C_j (row-major 3x3) between the previous joint frame and
    // this joint's Rz and the constant offset s_j (3) travelled in this joint's
    // frame; then the base position q0 (3).  A device array rather than kernarg
    // fields: the kernels stage it in LDS with a runtime-indexed loop, which on a
    // by-value kernarg struct costs a private copy of the whole struct.
    int32_t dh_off;
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
    // cooperative kernel only (ikpso_coop.h): G workgroups per swarm, NG groups
    unsigned long long* coop_slots;  // [NG][2][G][kCoopSlot(D)] granules {value, tag}: the chunk minima (zero, or
                                     // tags below coop_tag0 + 1, before the launch)
    int32_t* coop_error;      // set to 1 if a group wait timed out (device or pinned host memory;
                              // the kernels only write it)
    int32_t coop_g;
    int32_t coop_ng;
    int32_t coop_block;       // workgroup size (kCoopThreads<J>() or kCoopLatencyThreads)
    uint32_t coop_spin_limit; // polls before a group wait gives up (0: give up at the first unmet poll)
    unsigned long long* coop_timing;  // IKPSO_COOP_TIMING builds: [NG*G][4] cycle counts (else null)
    int32_t coop_linear;      // membership: 0 = XCD-aware (a group on one XCD, NG a multiple of 8),
                              // 1 = linear (group = workgroup / G: a latency group wider than an XCD)
    // The first exchange number of this launch: granule tags run tag0 + 1 ..
    // tag0 + exchanges, so granules a previous launch left (smaller tags) never
    // match and the slots need no clearing between launches (the per-frame call;
    // 0 with freshly zeroed slots otherwise).
    uint32_t coop_tag0;
    // Optional [B][P] copy of the generator states, written as each chunk loads
    // them (what a streaming re-run restarts from), or null.  Complete only when
    // every swarm is started in the launch's first round (the hosts pass it for
    // one swarm: a group that gives up never loads its later swarms).
    ikpso_rng_state* rng_snap;
};

// Streaming (state-in-HBM) kernels: one launch per PSO iteration over every
// chunk of every swarm.  Launch t (0 = init, 1..I = iterations, I+1 =
// finalize) writes its per-chunk argmin partials and the swarm's global-best
// state to slot t&1 and reads the previous launch's from slot (t-1)&1, so no
// workgroup ever reads what another workgroup of the same launch writes.
constexpr int kStreamChunk = 256;  // particles per workgroup (4 waves)

struct StreamIO {
    float* state;               // [B][3][D][P]: x | v | pbest planes (the reference's particles layout)
    float* pbf;                 // [B][P] local-best fitness
    uint32_t* rng;              // SoA [6][B*P] generator words (d, v0..v4)
    ikpso_rng_state* rng_aos;   // [B][P] caller/solver states: read at init, written at finalize
    uint32_t* pkey;             // [2][B][C] chunk-min keys
    int32_t* pidx;              // [2][B][C] chunk-min particle index
    float* pvec;                // [2][B][C][D] chunk winner's pbest
    uint32_t* gkey;             // [2][B] global-best key (0xFFFFFFFF before the first copy)
    int32_t* gidx;              // [2][B]
    float* gvec;                // [2][B][D] global-best vector
    const float* targets;       // [B][E][3] or null
    const float* start_pose;    // [B][D] or null
    float* out_angles;          // [B][D]
    float* out_fitness;         // [B] or null
    float* out_residual;        // [B] or null
    int64_t num_swarms;
    int32_t P;
    int32_t C;                  // chunks per swarm
    int32_t t;                  // launch index (see above)
    int32_t pad_;
};

}  // namespace ikpso
