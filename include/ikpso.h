/*
 * ikpso.h -- C ABI of the MI355X-native PSO inverse-kinematics solver.
 *
 * This is the drop-in boundary for the reference's solver hot path
 * (MadDevX/Inverse-Kinematics-PSO-Research, src/ = InverseKinematicsResearch/
 * InverseKinematicsResearch/).  Plain C types, plain pointers and sizes; no
 * torch or C++ types.  Every entry point returns an ikpso_status (0 = success,
 * mirroring cudaSuccess/hipSuccess: the reference's caller aborts its frame
 * loop on any non-zero value, src/Main.cpp:225-226).
 *
 * Memory: "device" pointers are HIP device allocations (hipMalloc) or managed
 * allocations (hipMallocManaged); "any" pointers may be host, managed or device
 * memory (copied with hipMemcpyDefault).  Stream: a hipStream_t passed as
 * void*; NULL = the legacy default stream.  Calls are stream-ordered; the
 * reference-compatible entry points additionally synchronise before returning,
 * as the reference does (src/kernel.cu:317-322).
 */
#ifndef IKPSO_H
#define IKPSO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IKPSO_ABI_VERSION 5

typedef int ikpso_status;
enum {
    IKPSO_OK = 0,
    IKPSO_ERR_INVALID_ARG = 1,   /* bad size, null pointer, bad node table */
    IKPSO_ERR_UNSUPPORTED = 2,   /* no compiled kernel for this chain / swarm size / kernel family */
    IKPSO_ERR_HIP = 3,           /* a HIP runtime call failed; see ikpso_last_hip_error() */
    IKPSO_ERR_NO_MEMORY = 4
};

/* Node types, same values as the reference's NodeType (src/Particle.h:10-15). */
enum { IKPSO_NODE_ORIGIN = 0, IKPSO_NODE_EFFECTOR = 1, IKPSO_NODE = 2 };

/* One node of the kinematic tree; byte-identical to the reference's NodeCUDA
 * (src/Particle.h:24-39, 88 bytes).  Node 0 is the origin; nodes 1..J are
 * 3-axis Euler-XYZ joints followed by a link of `length` along local +X
 * (src/kernel.cu:52-56); parent_index < own index (DFS order, src/Node.h:232-267). */
typedef struct ikpso_node {
    int32_t node_type;
    int32_t parent_index;
    float effector_weight;
    float position[3];        /* origin only */
    float rotation[3];        /* current pose = warm start + angle-term reference */
    float max_rotation[3];    /* clamp bounds, per Euler axis */
    float min_rotation[3];
    float length;
    float target_position[3]; /* effectors only */
    float target_rotation[3]; /* unused by the fitness (as in the reference) */
} ikpso_node;

/* XORWOW generator state with cuRAND's curandStateXORWOW layout (48 bytes),
 * so N * sizeof(curandState_t) allocations stay valid (src/Main.cpp:137). */
typedef struct ikpso_rng_state {
    uint32_t d;
    uint32_t v[5];
    int32_t boxmuller_flag;
    int32_t boxmuller_flag_double;
    float boxmuller_extra;
    uint32_t pad_;
    double boxmuller_extra_double;
} ikpso_rng_state;

/* PSOConfig (src/Particle.h:70-85): passed by value like the reference. */
typedef struct ikpso_pso_config {
    float inertia;
    float local;
    float global;
    int32_t iterations;
} ikpso_pso_config;

/* FitnessConfig (src/Particle.h:55-68). */
typedef struct ikpso_fitness_config {
    float angle_weight;
    float distance_weight;
    float error_threshold; /* never read, as in the reference */
} ikpso_fitness_config;

/* obj_t (src/BoxCollider.h:4-10): box edge lengths x, y, z (supportBox uses
 * +-x/2), centre, orientation quaternion (x, y, z, w). */
typedef struct ikpso_collider {
    float x, y, z;
    float pos[3];
    float pad_[2];
    float quat[4]; /* float4, 16-byte aligned in the reference */
} ikpso_collider;

/* Kernel family (ikpso_solver_desc.kernel; env IKPSO_KERNEL for ikpso_calculate_pso). */
enum {
    IKPSO_KERNEL_AUTO = 0,      /* resident when the swarm fits one workgroup, else cooperative, else streaming */
    IKPSO_KERNEL_RESIDENT = 1,  /* one workgroup per swarm, state on chip, one launch per batch */
    IKPSO_KERNEL_STREAMING = 2, /* state in HBM, one launch per iteration, any swarm size */
    IKPSO_KERNEL_COOP = 3       /* one swarm over G co-resident workgroups (G CUs), state on chip, one
                                   launch per batch; AUTO picks it for swarms above one workgroup when
                                   the chain has a specialised kernel and G <= CUs / 8 */
};

/* Arithmetic mode of the device kernels. */
enum {
    IKPSO_ARITH_FAST = 0,      /* closed-form 3x3 FK, FMA contraction (default); sin/cos on the
                                  transcendental unit when every clamp bound and rest angle of the
                                  chain lies within +-100 rad (the answers are clamped there), else a
                                  1-ulp polynomial.  A start pose (or the rest pose of the compat
                                  call) beyond +-100 rad inside such bounds is evaluated once, at
                                  initialisation, with the unit's larger error there (~1e-5 at 150 rad);
                                  every later evaluation is of clamped angles.  The resident and
                                  cooperative FAST kernels keep angles in revolutions (x / 2pi), so
                                  answers and dumped particles come back within 4 ulp of the radian
                                  values -- at 0 iterations the rest pose within 4 ulp, not bit for
                                  bit (REFERENCE returns it exactly) */
    IKPSO_ARITH_REFERENCE = 1  /* the reference's 4x4 operation order, no FMA contraction */
};

/* ---------------------------------------------------------------------------
 * Reference-compatible entry points (single swarm).
 * ------------------------------------------------------------------------- */

/* Replaces initGenerators (src/utility_kernels.cuh:33-47, declared at
 * src/Main.cpp:28): randoms[i] = curand_init(i, 0, 0).  randoms: device. */
ikpso_status ikpso_init_generators(ikpso_rng_state* randoms, int size, void* stream);

/* Generalised seeding: randoms[i] = curand_init(seed_base + i, 0, 0). */
ikpso_status ikpso_init_generators_seeded(ikpso_rng_state* randoms, int64_t count, uint64_t seed_base,
                                          void* stream);

/* Replaces calculatePSO (src/kernel.cu:279-327, declared at src/Main.cpp:29).
 *   particles [3][D][size] floats, device: SoA position / velocity / local best
 *             (src/kernel.cu:17-29); overwritten with the final swarm state.
 *   positions [4*J] floats, any: host-computed arm positions, read only when
 *             fit.distance_weight != 0, at slot (k-1)*4 for node k (src/kernel.cu:94-98);
 *             [4*(J+2)] read at slot (k+1)*4 with IKPSO_POSREF=node_slot (see IKPSO_FLAG_*).
 *   bests     [size] floats, device: final local-best fitness per particle.
 *   randoms   [size] states, device: consumed and advanced (persist across calls).
 *   chain     [node_count] nodes, any.  D = 3*(node_count-1).
 *   result    [D] floats, any: global-best joint angles (Coordinates).
 *   colliders [collider_count] obj_t, any: boxes of the collider term (src/kernel.cu:104-136):
 *             a particle whose node or link box intersects one (GJK) gets fitness FLT_MAX.
 * Synchronises `stream` before returning.  After the argument checks, an error the
 * caller's earlier HIP work left pending (unread by hipGetLastError) is returned
 * (IKPSO_ERR_HIP, ikpso_last_hip_error) and consumed up front, and nothing runs:
 * particles, bests, randoms and result are left untouched.  The reference returns
 * such an error too (its first cudaGetLastError check, src/kernel.cu:293-295), but
 * only after its init kernels have rewritten particles, bests and randoms.
 * ikpso_solver_create and ikpso_solve_batch take a pending error the same way
 * (a stale error from unrelated earlier work fails them; read it with
 * hipGetLastError first to avoid that). */
ikpso_status ikpso_calculate_pso(float* particles, const float* positions, float* bests,
                                 ikpso_rng_state* randoms, int size, const ikpso_node* chain, int node_count,
                                 ikpso_pso_config pso, ikpso_fitness_config fit, float* result,
                                 const ikpso_collider* colliders, int collider_count, void* stream);

/* ---------------------------------------------------------------------------
 * Batched API: B independent swarms (IK targets) per call, one launch.
 * ------------------------------------------------------------------------- */

typedef struct ikpso_solver ikpso_solver;

typedef struct ikpso_solver_desc {
    const ikpso_node* chain;  /* any; node table shared by every swarm */
    int32_t node_count;       /* J + 1 */
    int32_t particles;        /* P per swarm */
    ikpso_pso_config pso;
    ikpso_fitness_config fit;
    int32_t arith;            /* IKPSO_ARITH_* */
    int32_t kernel;           /* IKPSO_KERNEL_* */
    const float* positions;   /* any, [4*J] or NULL (distance term, as calculatePSO) */
    /* Optional soft joint-limit penalty (a new term; the reference only clamps):
     * fitness += limit_weight * sum_d max(0, x_d - soft_hi[d], soft_lo[d] - x_d)^2 */
    float limit_weight;
    float reserved1;
    const float* soft_lo;     /* any, [D] or NULL */
    const float* soft_hi;     /* any, [D] or NULL */
    /* Collider term, as calculatePSO's colliders/colliderCount (ABI >= 2). */
    const ikpso_collider* colliders; /* any, [collider_count] or NULL */
    int32_t collider_count;
    int32_t flags;            /* IKPSO_FLAG_* */
    /* Joint-axis mask (ABI >= 4; an extension -- the reference hard-wires three
     * Euler axes per node, src/kernel.cu:52-56,160-187): any, [node_count] or
     * NULL.  Bit c of axis_mask[k] set = Euler angle c of node k is a PSO
     * dimension; a clear bit locks that angle at the node's rotation[c] (no
     * draws, no update, no clamp; the angle term sees an exact zero).  Entry 0
     * (the origin) is ignored.  NULL = every axis free = the reference.  D, the
     * solver's dimension count, is then the number of free axes: start poses,
     * answers, soft limits and evaluate()'s angles carry those D values in node
     * order, axis order within a node.  FAST solves of a serial chain with a
     * tip effector and no distance/collider term run on the chain folded into
     * its free axes (one sincos per free angle; DH arms); see IKPSO_FLAG_NO_FOLD. */
    const uint8_t* axis_mask;
} ikpso_solver_desc;

/* ikpso_solver_desc.flags (env IKPSO_POSREF=node_slot for ikpso_calculate_pso). */
enum {
    /* Distance term with the reference's latent slot bug fixed (opt-in): the
     * reference reads node k's reference position from positions[(k-1)*4],
     * which FillPositions (src/Node.h:110-149) filled with node k-2's; with
     * this flag positions is [4*(J+2)] as FillPositions writes it and node k
     * reads slot k+1, its own.  Off: bit-compatible with the reference. */
    IKPSO_FLAG_POSREF_NODE_SLOT = 1,
    /* Solve a masked chain with the Euler kernels (locked axes skipped) even
     * where the folded form applies (ABI >= 4; comparisons and tests). */
    IKPSO_FLAG_NO_FOLD = 2
};

ikpso_status ikpso_solver_create(const ikpso_solver_desc* desc, ikpso_solver** out);
ikpso_status ikpso_solver_destroy(ikpso_solver* solver);

/* Allocate (or re-seed) the solver-owned generator states for `capacity`
 * swarms: state of local swarm b, particle i = curand_init(seed_base +
 * (first_swarm + b) * P + i, 0, 0).  first_swarm is the global index of local
 * swarm 0, so a batch sharded over ranks draws the same streams as one rank.
 * States persist across solve calls (like the reference's randoms buffer). */
ikpso_status ikpso_solver_seed(ikpso_solver* solver, int64_t capacity, uint64_t seed_base, int64_t first_swarm,
                               void* stream);

/* Solve `num_swarms` (<= capacity) swarms for `iterations` PSO iterations.
 *   targets    device, [B][E][3]: effector targets, effectors in node order.
 *   start_pose device, [B][D] or NULL (NULL: chain rotations).
 *   out_angles device [B][D]; out_fitness device [B]; out_residual device [B] or NULL
 *   (residual = sum over effectors of |p_e - t_e|, as checkDistance).
 * Stream-ordered; does not synchronise.  A solver handle owns one workspace:
 * calls on one handle must be ordered (one stream, or synchronised), not
 * concurrent.  The cooperative family needs its workgroups co-resident (one per
 * CU): the grid is checked against the occupancy query at launch, and if other
 * work on the device still keeps a group from assembling, its bounded wait
 * gives up (never a hang) and the swarms it had not finished get NaN angles,
 * fitness and residual -- until ikpso_solver_sync settles the solve. */
ikpso_status ikpso_solve_batch(ikpso_solver* solver, const float* targets, const float* start_pose,
                               int64_t num_swarms, int32_t iterations, float* out_angles, float* out_fitness,
                               float* out_residual, void* stream);

/* Settle the last solve_batch (ABI >= 3).  After a cooperative-family solve:
 * wait for it and, if a group gave up (the GPU shared with other work), restore
 * the generator states from the snapshot taken before the launch and re-run the
 * batch on the streaming kernels, which need no co-residency, so the outputs are
 * always a complete solve.  Returns at once after the other families.  The
 * buffers passed to that solve_batch must still be valid.  solve_batch settles a
 * pending solve itself before it launches the next one. */
ikpso_status ikpso_solver_sync(ikpso_solver* solver);
/* Solves of this handle / of the process that took the streaming fallback. */
int64_t ikpso_solver_fallbacks(const ikpso_solver* solver);
int64_t ikpso_coop_fallbacks(void);

/* Evaluate the device FK + fitness for n angle vectors (no PSO):
 *   angles device [n][D]; targets device [n][E][3] or NULL (chain targets);
 *   rest device [n][D] or NULL (chain rotations); out_fitness device [n] or NULL;
 *   out_positions device [n][J][3] or NULL (world position of nodes 1..J).
 *   D = free dimensions (the axis mask); locked angles at the chain's rotation.
 *   Always the Euler form of the chain (a folded FAST solver's answers agree
 *   with it within the FAST tolerance). */
ikpso_status ikpso_solver_evaluate(ikpso_solver* solver, const float* angles, const float* targets,
                                   const float* rest, int64_t n, float* out_fitness, float* out_positions,
                                   void* stream);

/* Copy the generator states of local swarms [first_swarm, first_swarm + count)
 * (P states each, swarm-major, 48-byte curandState layout) into dst (any memory,
 * count * P states), after settling a pending solve (ABI >= 5).  Synchronises
 * `stream`.  The parity tests compare them with the oracle's: the draw count of
 * every particle (D at init, 3 D per iteration) is integer work, bit-exact. */
ikpso_status ikpso_solver_generator_states(ikpso_solver* solver, int64_t first_swarm, int64_t count, void* dst,
                                           void* stream);

/* Introspection.  dof = D, the free dimensions. */
int ikpso_solver_dof(const ikpso_solver* solver);
int ikpso_solver_effectors(const ikpso_solver* solver);
/* Colliders the solver's kernels test: those of the descriptor's colliders that lie
 * within the arm's reach of some node (one beyond it can never touch the arm, so it
 * can never change a fitness); with none left the chain is solved by the kernels
 * without the collider term.  The environment variable IKPSO_KEEP_FAR_COLLIDERS=1
 * keeps every collider. */
int ikpso_solver_collider_count(const ikpso_solver* solver);
/* Name of the kernel variant the solver dispatches to (family / topology); after a
 * solve_batch that AUTO routed to the cooperative latency variant (a few swarms),
 * that variant's name until the next solve. */
const char* ikpso_solver_kernel_name(const ikpso_solver* solver);

int ikpso_abi_version(void);
/* Hash of the sources the library was built from (csrc/ *.h *.hip *.cpp Makefile,
 * include/ *.h; ABI >= 5), plus "+" and a hash of the extra compiler flags of a
 * variant build.  The Python loader compares it with the tree it runs from. */
const char* ikpso_build_id(void);
const char* ikpso_status_string(ikpso_status status);
int ikpso_last_hip_error(void);

#ifdef __cplusplus
}
#endif

#endif /* IKPSO_H */
