// ikpso_kernels.h -- host-side view of the kernel library: the parsed chain,
// launch entry points and their parameter blocks.
#pragma once

#include <hip/hip_runtime.h>

#include <string.h>

#include <string>
#include <vector>

#include "ikpso.h"
#include "ikpso_collide.h"
#include "ikpso_params.h"

// Experiment builds (tools/build_variants.sh) compile a subset of topologies.
// DH_ONLY: the folded chains and the 6-14-joint serial chains they fold from.
#if defined(IKPSO_EXPERIMENT_REF7_ONLY)
#define IKPSO_WITH_REF7 1
#define IKPSO_WITH_SERIAL20 0
#define IKPSO_WITH_OTHERS 0
#define IKPSO_WITH_DH 0
#elif defined(IKPSO_EXPERIMENT_SERIAL20_ONLY)
#define IKPSO_WITH_REF7 0
#define IKPSO_WITH_SERIAL20 1
#define IKPSO_WITH_OTHERS 0
#define IKPSO_WITH_DH 0
#elif defined(IKPSO_EXPERIMENT_REF7_SERIAL20)
#define IKPSO_WITH_REF7 1
#define IKPSO_WITH_SERIAL20 1
#define IKPSO_WITH_OTHERS 0
#define IKPSO_WITH_DH 0
#elif defined(IKPSO_EXPERIMENT_DH_ONLY)
#define IKPSO_WITH_REF7 0
#define IKPSO_WITH_SERIAL20 0
#define IKPSO_WITH_OTHERS 0
#define IKPSO_WITH_DH 1
#else
#define IKPSO_WITH_REF7 1
#define IKPSO_WITH_SERIAL20 1
#define IKPSO_WITH_OTHERS 1
#define IKPSO_WITH_DH 1
#endif

namespace ikpso {

// Ref7: the reference scene's tree with effectors on nodes 5..7; SerialTip:
// serial chain with a single tip effector; Generic: anything else.
// DH: a serial chain with a tip effector folded into its free angles (TopoDH;
// built from a masked chain by the API layer, FAST arithmetic).
enum class TopoKind { Ref7, SerialTip, Generic, DH };

// The chain as the kernels need it, parsed once from the caller's node table.
struct ChainHost {
    int J = 0;  // joints = node_count - 1
    int E = 0;  // effectors
    TopoKind topo = TopoKind::Generic;
    std::vector<int> parent, eff_slot;
    std::vector<float> len, eff_w, lo, hi, rest, tgt0;
    // [posref 4J | soft_lo 3J | soft_hi 3J | collider records 16*num_coll | near limits J*num_coll |
    //  TopoDH constants] (host copy)
    std::vector<float> aux;
    const float* aux_dev = nullptr;  // device copy, owned by the solver / call
    float m0[12] = {};
    float w = 0, c1 = 0, c2 = 0, aw_j = 0, dw_j = 0, lim_w = 0;
    bool use_posref = false, use_penalty = false;
    bool uniform_bounds = false;  // every angle has clamp bounds lo[0], hi[0]
    bool unit_rev_bounds = false; // ... and they are [0, 1] in revolutions (kTermUnitBounds): [0, 2pi]
    bool ordered_bounds = false;  // ... and finite with lo <= hi (REFERENCE uniform builds: median clamp)
    bool sym_penalty = false;     // soft limits symmetric and within a revolution of the clamp (kTermSymPenalty)
    int num_coll = 0;             // colliders (obj_t) of the scene within the arm's reach (parse_chain)
    int colliders_dropped = 0;    // ... and those left out, beyond it
    size_t coll_off = 0;          // float offset of the collider records in aux
    size_t coll_lim_off = 0;      // ... of near_collider's squared limits [J][num_coll] (after the records)
    size_t coll_box_off = 0;      // ... of the colliders as oriented boxes [num_coll][16] (after the limits)
    bool coll_obb = true;         // every collider's quaternion is a rotation (|q| = 1 to 1e-5): the FAST
                                  // builds may test it as an oriented box (kFastSat); else they take GJK
    // joint-axis mask over the kernel's dimensions (all set: no mask) and the
    // number of free dimensions, which is the API's D
    uint64_t free_mask = 0;
    int dfree = 0;
    bool masked = false;          // some Euler angle is locked: runtime-term kernels only
    // a free angle's clamp bound or rest value lies beyond kHwTrigMaxAbs: FAST
    // solves take the polynomial sin/cos (the collider builds, with no collider)
    bool poly_trig = false;
    size_t dh_off = 0;            // TopoDH constants in aux (ChainConsts::dh_off), 12 J + 4 floats
    int dof() const { return dfree; }
    int kernel_dims() const { return topo == TopoKind::DH ? J : 3 * J; }
};

// Evaluate-kernel parameters.
struct EvalIO {
    const float* angles;   // [n][D]
    const float* targets;  // [n][E][3] or null (chain targets)
    const float* rest;     // [n][D] or null (chain rotations)
    float* out_fitness;    // [n] or null
    float* out_positions;  // [n][J][3] or null
    int64_t n;
};

// Threads per workgroup the resident kernel is compiled for, by the kernel's
// dimension count D: 1024 lanes (16 waves, 4 per SIMD, <= 128 VGPRs) while
// x/v/pbest of one particle fit (D <= 30), 256 lanes (one wave per SIMD, up to
// 512 VGPRs) for long chains.
template <int D>
__host__ __device__ constexpr int kResidentMaxThreads()
{
    return D <= 30 ? 1024 : 256;
}

// Threads per workgroup of the cooperative kernel, and its workgroups per CU:
// the resident kernel's 1024 for short chains, one per CU; for long ones 256
// lanes (one wave per SIMD, 60 KiB of local bests at D = 60) and TWO workgroups
// per CU, each a chunk of a different swarm -- 2 waves per SIMD (<= 256 VGPRs)
// as with one 512-lane chunk, but one swarm's argmin barrier and cross-CU
// hand-off hide under the other swarm's step.
template <int D>
__host__ __device__ constexpr int kCoopThreads()
{
    return D <= 30 ? 1024 : 256;
}
template <int D>
__host__ __device__ constexpr int kCoopBlocksPerCU()
{
    return D <= 30 ? 1 : 2;
}

#ifndef IKPSO_COOP_TIMING
#define IKPSO_COOP_TIMING 0  // measurement builds: per-workgroup cycles in the step and in the hand-off
#endif
// REFERENCE arithmetic on the reference scene with uniform ordered bounds gets its
// own resident build (no runtime term tests, median clamp); 0: the runtime-term
// build as before (A/B timing).
#ifndef IKPSO_REF_UNIFORM_BUILD
#define IKPSO_REF_UNIFORM_BUILD 1
#endif
// The cooperative latency variant with its generators on separate waves
// (k_swarm_coop_split, ikpso_coop.h); 0 builds the unsplit one (A/B timing).
#ifndef IKPSO_SPLIT_GEN
#define IKPSO_SPLIT_GEN 1
#endif
// Quads of an iteration's draw block the generator waves write beside the step
// (the rest during the hand-off); -1: half.
#ifndef IKPSO_SPLIT_QA
#define IKPSO_SPLIT_QA -1
#endif

// IKPSO_COLLIDE_STATS builds: the device counters the collider term adds to (null otherwise).
unsigned long long* collide_stats_buffer();

// Published record of one chunk, in 8-byte granules {value, tag}: the key, then
// the D floats of the chunk winner's local best; padded to a 128-B multiple.
__host__ __device__ constexpr int kCoopSlot(int D) { return ((D + 1 + 15) / 16) * 16; }
// Default bound on a cooperative group wait (polls of ~1 us each): seconds,
// against ~2 us per exchange when the group is co-resident.
// IKPSO_COOP_SPIN_LIMIT overrides it (0 forces the give-up path: fallback tests).
constexpr uint32_t kCoopSpinLimit = 1u << 22;
// Latency variant of the cooperative kernel (few swarms): 256-lane chunks,
// one wave per SIMD, a swarm of 1024 over 4 CUs.
constexpr int kCoopLatencyThreads = 256;
// Largest |angle| the FAST kernels hand to the transcendental unit's v_sin/v_cos
// (which take x / 2pi): tools/probes/trig_probe.hip measures the max abs error
// at 4.8e-7 on [0, 2pi] and 7.0e-6 on [-100, 100] (the fp32 rounding of x / 2pi
// grows with |x|).  Chains whose clamp bounds or rest angles reach beyond it
// solve with the 1-ulp polynomial instead (ChainHost::poly_trig).
constexpr float kHwTrigMaxAbs = 100.0f;
// The transcendental unit's v_sin_f32 / v_cos_f32 round toward zero more often
// than not: over a revolution e_sin = -eps sin, e_cos = -eps cos with eps =
// 3.23e-8 (tools/probes/hwtrig_bias.hip, profiles/r05/hwtrig_bias.txt), so each
// plane rotation built from them shrinks the in-plane part of the vector it turns
// by eps.  A link vector passes the 3 plane rotations of every node from the root
// to its own node (in the frame-composition and the tip-backward forms alike:
// the rotations' product is the same); with an isotropic in-plane share of 2/3
// that is an expected shrink of 2 depth(k) eps for link k -- 7.7e-7 of the reach
// of config 5's 20-joint chain, a median +1.4e-6 of its final fitness (round 5's
// strict sign test: 83 worse / 44 better than the oracle).  The FAST kernels on
// the transcendental unit therefore use link lengths scaled up by that much
// (ChainConsts::len_hw; fp64, rounded once): the strict count became 55 / 66
// (profiles/r06/hwtrig_comp.txt).  Per value no fp32 correction exists (1 + eps
// rounds back to 1); per link the scaled length is representable.
constexpr double kHwTrigAmplitudeBias = 3.23e-8;
template <int J>
ChainConsts<J> make_consts(const ChainHost& h)
{
    ChainConsts<J> c;
    memset(&c, 0, sizeof(c));
    int depth[J + 1];
    depth[0] = 0;
    for (int k = 1; k <= J; ++k) depth[k] = (h.parent[k] > 0 ? depth[h.parent[k]] : 0) + 1;
    for (int k = 0; k <= J; ++k) {
        c.len[k] = h.len[k];
        c.len_hw[k] = k ? (float)((double)h.len[k] * (1.0 + 2.0 * depth[k] * kHwTrigAmplitudeBias)) : h.len[k];
        c.eff_w[k] = h.eff_w[k];
        c.eff_slot[k] = h.eff_slot[k];
        c.parent[k] = h.parent[k];
    }
    for (int d = 0; d < 3 * J; ++d) {
        c.lo[d] = h.lo[d];
        c.hi[d] = h.hi[d];
        c.rest[d] = h.rest[d];
        c.tgt0[d] = h.tgt0[d];
    }
    for (int i = 0; i < 12; ++i) c.m0[i] = h.m0[i];
    c.aux = h.aux_dev;
    c.w = h.w;
    c.c1 = h.c1;
    c.c2 = h.c2;
    c.wq = h.w * 0x1p-32f;
    c.c1q = h.c1 * 0x1p-32f;
    c.c2q = h.c2 * 0x1p-32f;
    c.wh = h.w * 0x1p-33f;
    c.c1h = h.c1 * 0x1p-33f;
    c.c2h = h.c2 * 0x1p-33f;
    c.aw_j = h.aw_j;
    c.dw_j = h.dw_j;
    c.lim_w = h.lim_w;
    c.aw_rev = h.aw_j * 39.4784176043574344f;  // (2 pi)^2
    c.lim_rev = h.lim_w * 39.4784176043574344f;
    c.rlo = h.lo.empty() ? 0.0f : h.lo[0] * 0.159154943091895336f;
    c.rhi = h.hi.empty() ? 0.0f : h.hi[0] * 0.159154943091895336f;
    c.use_posref = h.use_posref ? 1 : 0;
    c.use_penalty = h.use_penalty ? 1 : 0;
    c.num_eff = h.E;
    c.num_coll = h.num_coll;
    c.coll = h.num_coll && h.aux_dev ? reinterpret_cast<const CollRec*>(h.aux_dev + h.coll_off) : nullptr;
    c.coll_lim = h.num_coll && h.aux_dev ? h.aux_dev + h.coll_lim_off : nullptr;
    c.coll_box = h.num_coll && h.aux_dev ? h.aux_dev + h.coll_box_off : nullptr;
    c.coll_stats = collide_stats_buffer();
    c.free_mask = h.free_mask;
    c.dfree = h.dfree;
    c.dh_off = (int32_t)h.dh_off;
    return c;
}

hipError_t launch_init_generators(ikpso_rng_state* st, int64_t count, uint64_t seed_base, hipStream_t stream);
hipError_t launch_resident(const ChainHost& ch, int mode, const SwarmIO& io, hipStream_t stream);
hipError_t launch_stream(const ChainHost& ch, int mode, const StreamIO& io, int iterations, hipStream_t stream);
size_t stream_workspace_bytes(int64_t B, int P, int D, bool with_state);
hipError_t launch_evaluate(const ChainHost& ch, int mode, const EvalIO& io, hipStream_t stream);
// Cooperative resident kernel (ikpso_coop.h): io.coop_* describe the grid and workspace.
hipError_t launch_coop(const ChainHost& ch, int mode, const SwarmIO& io, hipStream_t stream);
// Co-resident workgroups per CU of the cooperative kernel, CU count, threads per workgroup.
struct CoopGeometry {
    int threads = 0, blocks_per_cu = 0, cus = 0;
    bool latency_variant = false;  // a kCoopLatencyThreads build exists for this chain
};
bool coop_geometry(const ChainHost& ch, int mode, CoopGeometry* g);
size_t coop_workspace_bytes(int ng, int G, int D, int block);
bool coop_latency_split(const ChainHost& ch);  // latency variant with generator waves
int resident_max_threads(const ChainHost& ch);
bool chain_supported(const ChainHost& ch);
std::string kernel_name(const ChainHost& ch, int family);  // IKPSO_KERNEL_*

}  // namespace ikpso
