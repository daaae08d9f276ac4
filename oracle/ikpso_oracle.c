/*
 * ikpso_oracle.c -- CPU restatement of the reference PSO inverse-kinematics
 * hot path.  TEST INFRASTRUCTURE ONLY: this file is the parity checker for the
 * HIP product path and the "port" CPU baseline timed by bench.py.  Nothing in
 * the product (inverse-kinematics-pso-research_amd/) links, loads or calls it.
 *
 * Reference: MadDevX/Inverse-Kinematics-PSO-Research,
 *   src/ = InverseKinematicsResearch/InverseKinematicsResearch/
 * The reference cannot be built in this container (it needs the CUDA toolkit,
 * cuRAND and Thrust headers, none of which exist here), so this is a
 * restatement, written from the reference's behaviour:
 *
 *   - getParticleIndex            src/kernel.cu:17-29        -> pidx()
 *   - updateChainMatrices         src/kernel.cu:31-62        -> orc_chain_matrices()
 *   - createMatrix/multiplyMatrices/translateMatrix/rotateMatrixAlong{X,Y,Z}/
 *     rotateEuler/clamp           src/matrix_operations.cuh:5-38,123-190
 *   - calculateDistance (fitness) src/kernel.cu:64-151       -> orc_fitness_soa()
 *   - simulateParticlesKernel     src/kernel.cu:153-189      -> step loop in orc_calculate_pso()
 *   - initLocalBests/updateLocalBests src/kernel.cu:191-221
 *   - initParticlesKernel         src/kernel.cu:223-266
 *   - updateGlobalBestCoordsKernel src/kernel.cu:268-277
 *   - calculatePSO host driver    src/kernel.cu:279-327      -> orc_calculate_pso()
 *   - randInitKernel/initGenerators src/utility_kernels.cuh:21-47 -> orc_init_generators()
 *   - EffectorNode::calculateDistance / checkDistance src/Node.h:421-429,
 *     src/Main.cpp:290-298       -> orc_residual()
 *   - the collider (GJK) block of calculateDistance src/kernel.cu:104-136 -> ikpso_gjk.c
 *
 * Third-party arithmetic restated from its published algorithm (not vendored
 * in the reference): cuRAND XORWOW (curand_init(seed,0,0), curand(),
 * curand_uniform()) from the CUDA 10.1 toolkit's curand_kernel.h, and
 * thrust::min_element (first minimum, operator<).
 *
 * Arithmetic: plain IEEE fp32, evaluated in the reference's operation order,
 * compiled with -ffp-contract=off (no FMA).  sinf/cosf: the reference calls
 * CUDA's precise sinf/cosf (<= 2 ulp, src/matrix_operations.cuh:136-161; not
 * available here); they are restated as the correctly rounded values
 * (float)sin((double)x), which glibc's own sinf/cosf miss by 1 ulp on ~1.4% of
 * arguments in [-7, 7].  The three
 * curand_uniform() calls in one expression (src/kernel.cu:164-166) are drawn
 * left to right (r1, r2, r3).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ types */

/* curandStateXORWOW layout (48 bytes). */
typedef struct {
    uint32_t d;
    uint32_t v[5];
    int32_t boxmuller_flag;
    int32_t boxmuller_flag_double;
    float boxmuller_extra;
    uint32_t pad_;
    double boxmuller_extra_double;
} orc_rng;

/* NodeCUDA layout (src/Particle.h:24-39), 88 bytes. */
typedef struct {
    int32_t node_type; /* 0 origin, 1 effector, 2 node (src/Particle.h:10-15) */
    int32_t parent_index;
    float effector_weight;
    float position[3];
    float rotation[3];
    float max_rotation[3];
    float min_rotation[3];
    float length;
    float target_position[3];
    float target_rotation[3];
} orc_node;

enum { ORC_ORIGIN = 0, ORC_EFFECTOR = 1, ORC_NODE = 2 };

typedef struct { float c[16]; } mat4; /* row-major, cells[col + 4*row] */

/* correctly rounded fp32 sin/cos (see header) */
static inline float sin_cr(float x) { return (float)sin((double)x); }
static inline float cos_cr(float x) { return (float)cos((double)x); }

int orc_sizeof_rng(void) { return (int)sizeof(orc_rng); }
int orc_sizeof_node(void) { return (int)sizeof(orc_node); }

/* ---------------------------------------------------------------- XORWOW */

void orc_curand_init(uint64_t seed, orc_rng* s)
{
    uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    s->d = 6615241u + t1 + t0;
    s->v[0] = 123456789u + t0;
    s->v[1] = 362436069u ^ t0;
    s->v[2] = 521288629u + t1;
    s->v[3] = 88675123u ^ t1;
    s->v[4] = 5783321u + t0;
    s->boxmuller_flag = 0;
    s->boxmuller_flag_double = 0;
    s->boxmuller_extra = 0.0f;
    s->pad_ = 0;
    s->boxmuller_extra_double = 0.0;
    /* subsequence = 0 and offset = 0: no skip-ahead */
}

uint32_t orc_curand(orc_rng* s)
{
    uint32_t t = s->v[0] ^ (s->v[0] >> 2);
    s->v[0] = s->v[1];
    s->v[1] = s->v[2];
    s->v[2] = s->v[3];
    s->v[3] = s->v[4];
    s->v[4] = (s->v[4] ^ (s->v[4] << 4)) ^ (t ^ (t << 1));
    s->d += 362437u;
    return s->v[4] + s->d;
}

float orc_curand_uniform(orc_rng* s)
{
    uint32_t x = orc_curand(s);
    return (float)x * 2.3283064e-10f + (2.3283064e-10f / 2.0f);
}

/* initGenerators: curand_init(i, 0, 0, &randoms[i]) (src/utility_kernels.cuh:21-31),
 * generalised with a seed base: seed = seed_base + i. */
void orc_init_generators(orc_rng* randoms, int64_t size, uint64_t seed_base)
{
    for (int64_t i = 0; i < size; i++) orc_curand_init(seed_base + (uint64_t)i, &randoms[i]);
}

/* Advance `count` states by n draws each.  The v[5] recurrence of orc_curand is
 * linear over GF(2), so n steps are one 160x160 bit matrix A^n (built by
 * squaring; column j = A^n applied to unit state e_j, 5 words per column);
 * d is a plain counter, d += n * 362437.  Equivalent to n orc_curand calls
 * (tests/test_oracle.py checks it against the stepped loop).  Used to replay
 * the reference's recorded frame sequence: every calculatePSO call consumes a
 * fixed D + 3*D*I draws per particle, whatever the pose. */
typedef struct { uint32_t col[160][5]; } orc_gf2;

static void gf2_apply(const orc_gf2* m, const uint32_t in[5], uint32_t out[5])
{
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int j = 0; j < 160; j++)
        if ((in[j >> 5] >> (j & 31)) & 1u)
            for (int w = 0; w < 5; w++) r[w] ^= m->col[j][w];
    memcpy(out, r, sizeof(r));
}

static void gf2_mul(const orc_gf2* a, const orc_gf2* b, orc_gf2* out) /* out = a * b */
{
    orc_gf2 t;
    for (int j = 0; j < 160; j++) gf2_apply(a, b->col[j], t.col[j]);
    *out = t;
}

void orc_skipahead(orc_rng* states, int64_t count, uint64_t n)
{
    orc_gf2* base = (orc_gf2*)malloc(sizeof(orc_gf2));
    orc_gf2* acc = (orc_gf2*)malloc(sizeof(orc_gf2));
    for (int j = 0; j < 160; j++) { /* base = A (one step), acc = identity */
        orc_rng u;
        memset(&u, 0, sizeof(u));
        u.v[j >> 5] = 1u << (j & 31);
        orc_curand(&u);
        memcpy(base->col[j], u.v, sizeof(u.v));
        memset(acc->col[j], 0, sizeof(acc->col[j]));
        acc->col[j][j >> 5] = 1u << (j & 31);
    }
    for (uint64_t e = n; e; e >>= 1) {
        if (e & 1u) gf2_mul(base, acc, acc);
        if (e >> 1) gf2_mul(base, base, base);
    }
    const uint32_t dstep = (uint32_t)(n * 362437u);
    for (int64_t i = 0; i < count; i++) {
        gf2_apply(acc, states[i].v, states[i].v);
        states[i].d += dstep;
    }
    free(base);
    free(acc);
}

/* fill out[n] with uniforms drawn from one state (for RNG known-answer tests) */
void orc_uniform_stream(orc_rng* s, float* out, int n)
{
    for (int i = 0; i < n; i++) out[i] = orc_curand_uniform(s);
}

/* --------------------------------------------------------- 4x4 matrix ops */

static mat4 m_create(float f)
{
    mat4 m;
    for (int i = 0; i < 16; i++) m.c[i] = 0.0f;
    for (int i = 0; i < 4; i++) m.c[i + 4 * i] = f;
    return m;
}

static mat4 m_mul(mat4 l, mat4 r)
{
    mat4 o = m_create(0.0f);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            float sum = 0.0f;
            for (int x = 0; x < 4; x++) sum += l.c[x + j * 4] * r.c[x * 4 + i];
            o.c[i + j * 4] = sum;
        }
    return o;
}

static mat4 m_translate(mat4 l, float x, float y, float z)
{
    mat4 m = m_create(1.0f);
    m.c[3] = x;
    m.c[7] = y;
    m.c[11] = z;
    return m_mul(l, m);
}

static mat4 m_rot_x(mat4 l, float a)
{
    mat4 m = m_create(1.0f);
    m.c[5] = cos_cr(a);
    m.c[6] = -sin_cr(a);
    m.c[9] = sin_cr(a);
    m.c[10] = cos_cr(a);
    return m_mul(l, m);
}

static mat4 m_rot_y(mat4 l, float a)
{
    mat4 m = m_create(1.0f);
    m.c[0] = cos_cr(a);
    m.c[2] = sin_cr(a);
    m.c[8] = -sin_cr(a);
    m.c[10] = cos_cr(a);
    return m_mul(l, m);
}

static mat4 m_rot_z(mat4 l, float a)
{
    mat4 m = m_create(1.0f);
    m.c[0] = cos_cr(a);
    m.c[1] = -sin_cr(a);
    m.c[4] = sin_cr(a);
    m.c[5] = cos_cr(a);
    return m_mul(l, m);
}

static mat4 m_rot_euler(mat4 l, float x, float y, float z)
{
    l = m_rot_x(l, x);
    l = m_rot_y(l, y);
    l = m_rot_z(l, z);
    return l;
}

static float clampf_ref(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }

/* --------------------------------------------------- particle SoA indexing */

/* getParticleIndex (src/kernel.cu:17-29): prop 0 = position, 1 = velocity, 2 = localBest */
static inline int64_t pidx(int64_t count, int64_t i, int prop, int d, int dof)
{
    return i + count * d + (int64_t)prop * count * dof;
}

/* ------------------------------------------------------------- FK/fitness */

/* updateChainMatrices with the particle's angles given contiguously (angles[3*(k-1)+c]). */
void orc_chain_matrices(const orc_node* chain, int node_count, const float* angles, float* out16)
{
    mat4 m = m_create(1.0f);
    m = m_translate(m, chain[0].position[0], chain[0].position[1], chain[0].position[2]);
    m = m_rot_euler(m, chain[0].rotation[0], chain[0].rotation[1], chain[0].rotation[2]);
    memcpy(out16, m.c, sizeof(m.c));
    for (int k = 1; k < node_count; k++) {
        const float* a = angles + 3 * (k - 1);
        mat4 t = m_create(1.0f);
        t = m_rot_euler(t, a[0], a[1], a[2]);
        t = m_translate(t, chain[k].length, 0.0f, 0.0f);
        mat4 p;
        memcpy(p.c, out16 + 16 * chain[k].parent_index, sizeof(p.c));
        m = m_mul(p, t);
        memcpy(out16 + 16 * k, m.c, sizeof(m.c));
    }
}

static inline float msq3(float x, float y, float z) { return (x * x) + (y * y) + (z * z); }
static inline float msq4(float x, float y, float z, float w) { return (x * x) + (y * y) + (z * z) + (w * w); }

/* Optional soft joint-limit penalty -- an EXTENSION (BASELINE config 5), not in
 * the reference (which only clamps): f += limit_weight * sum_d over_d^2,
 * over_d = max(x_d - soft_hi_d, soft_lo_d - x_d, 0), summed in d order. */
typedef struct {
    float limit_weight;
    const float* soft_lo;
    const float* soft_hi;
    /* collider term (src/kernel.cu:104-136; ikpso_gjk.c): obj_t[collider_count] */
    const void* colliders;
    int collider_count;
    /* Joint-axis mask -- an EXTENSION, not in the
     * reference: axis_mask[k] (k = 1..J; entry 0 ignored) has bit c set when
     * Euler angle c of node k is a PSO dimension.  A locked axis keeps the
     * node's rotation[c] (its rest value) and takes no draws and no update; the
     * particle state, the draws, the clamp, the soft penalty, start poses and
     * results cover the D free dimensions only, in node order, axis order
     * within a node.  The fitness is the reference's calculateDistance of the
     * full Euler vector (locked entries add exact zeros to the angle term).
     * NULL = every axis free = the reference. */
    const uint8_t* axis_mask;
} orc_extra;

/* Free-dimension map of a chain: fd[d] = Euler index 3*(k-1)+c of free
 * dimension d; returns D. */
static int free_dims(const orc_extra* ex, int node_count, int* fd)
{
    int D = 0;
    for (int k = 1; k < node_count; k++)
        for (int c = 0; c < 3; c++)
            if (!ex || !ex->axis_mask || ((ex->axis_mask[k] >> c) & 1)) fd[D++] = 3 * (k - 1) + c;
    return D;
}

/* ikpso_gjk.c */
int orc_node_collides(const float* node, const float* parent, float length, const void* colliders, int count);

/* angles: the full Euler vector; soft_lo/soft_hi: per free dimension */
static float penalty_term(const orc_extra* pen, const float* angles, int node_count)
{
    int fd[3 * 64];
    const int D = free_dims(pen, node_count, fd);
    float p = 0.0f;
    for (int d = 0; d < D; d++) {
        const float a = angles[fd[d]];
        float over = fmaxf(fmaxf(a - pen->soft_hi[d], pen->soft_lo[d] - a), 0.0f);
        p = p + over * over;
    }
    return pen->limit_weight * p;
}

/* Full Euler vector of a chain from its free dimensions (locked axes at rest). */
static void expand_angles(const orc_node* chain, int node_count, const orc_extra* ex, const float* x, float* full)
{
    int fd[3 * 64];
    const int D = free_dims(ex, node_count, fd);
    for (int k = 1; k < node_count; k++)
        for (int c = 0; c < 3; c++) full[3 * (k - 1) + c] = chain[k].rotation[c];
    for (int d = 0; d < D; d++) full[fd[d]] = x[d];
}

static float fitness_pen(const orc_node* chain, int node_count, const float* positions, const float* angles,
                         float angle_weight, float distance_weight, const orc_extra* pen);

/* calculateDistance (src/kernel.cu:64-151) with colliderCount = 0 (orc_fitness_ex: any).
 * angles contiguous [D]; positions = host-filled arm positions (read at slot (ind-1)*4). */
float orc_fitness(const orc_node* chain, int node_count, const float* positions, const float* angles,
                  float angle_weight, float distance_weight)
{
    return fitness_pen(chain, node_count, positions, angles, angle_weight, distance_weight, NULL);
}

float orc_fitness_ex(const orc_node* chain, int node_count, const float* positions, const float* angles,
                     float angle_weight, float distance_weight, float limit_weight, const float* soft_lo,
                     const float* soft_hi, const void* colliders, int collider_count)
{
    orc_extra pen = {limit_weight, soft_lo, soft_hi, colliders, collider_count, NULL};
    return fitness_pen(chain, node_count, positions, angles, angle_weight, distance_weight, &pen);
}

static float fitness_pen(const orc_node* chain, int node_count, const float* positions, const float* angles,
                         float angle_weight, float distance_weight, const orc_extra* pen)
{
    const int dof = 3 * (node_count - 1);
    float rot_diff = 0.0f, pos_diff = 0.0f, distance = 0.0f;
    float mats[64 * 16];
    float* mp = node_count <= 64 ? mats : (float*)malloc(sizeof(float) * 16 * node_count);
    orc_chain_matrices(chain, node_count, angles, mp);
    for (int ind = 1; ind < node_count; ind++) {
        const float* a = angles + 3 * (ind - 1);
        rot_diff = rot_diff + msq3(chain[ind].rotation[0] - a[0], chain[ind].rotation[1] - a[1],
                                   chain[ind].rotation[2] - a[2]);
        const float* M = mp + 16 * ind;
        /* collider block (src/kernel.cu:104-136): any hit -> FLT_MAX */
        if (pen && pen->collider_count > 0 &&
            orc_node_collides(M, mp + 16 * chain[ind].parent_index, chain[ind].length, pen->colliders,
                              pen->collider_count)) {
            if (mp != mats) free(mp);
            return FLT_MAX;
        }
        /* multiplyMatByVec(model, (0,0,0,1)) */
        float px = M[0] * 0.0f + M[1] * 0.0f + M[2] * 0.0f + M[3] * 1.0f;
        float py = M[4] * 0.0f + M[5] * 0.0f + M[6] * 0.0f + M[7] * 1.0f;
        float pz = M[8] * 0.0f + M[9] * 0.0f + M[10] * 0.0f + M[11] * 1.0f;
        float pw = M[12] * 0.0f + M[13] * 0.0f + M[14] * 0.0f + M[15] * 1.0f;
        if (distance_weight != 0.0f && positions) {
            /* reads slot (ind-1)*4 exactly as the reference does (src/kernel.cu:94-98) */
            const float* ap = positions + (ind - 1) * 4;
            pos_diff += msq4(px - ap[0], py - ap[1], pz - ap[2], pw - ap[3]);
        }
        if (chain[ind].node_type == ORC_EFFECTOR) {
            float t = msq3(px - chain[ind].target_position[0], py - chain[ind].target_position[1],
                           pz - chain[ind].target_position[2]);
            distance = distance + t * chain[ind].effector_weight;
        }
    }
    if (mp != mats) free(mp);
    const float jn = (float)(dof / 3);
    float f = distance + distance_weight / jn * pos_diff + angle_weight / jn * rot_diff;
    if (pen && pen->limit_weight != 0.0f && pen->soft_lo && pen->soft_hi) f = f + penalty_term(pen, angles, node_count);
    return f;
}

/* calculateDistance of a masked chain: angles = the D free dimensions. */
float orc_fitness_mask(const orc_node* chain, int node_count, const float* positions, const float* angles,
                       float angle_weight, float distance_weight, float limit_weight, const float* soft_lo,
                       const float* soft_hi, const void* colliders, int collider_count, const uint8_t* axis_mask)
{
    orc_extra pen = {limit_weight, soft_lo, soft_hi, colliders, collider_count, axis_mask};
    float full[3 * 64];
    if (node_count > 64) return NAN;
    expand_angles(chain, node_count, &pen, angles, full);
    return fitness_pen(chain, node_count, positions, full, angle_weight, distance_weight, &pen);
}

/* particles: [3][D][count] over the free dimensions */
static float fitness_soa(const orc_node* chain, int node_count, const float* positions, const float* particles,
                         int64_t count, int64_t i, float aw, float dw, const orc_extra* pen)
{
    int fd[3 * 64];
    const int D = free_dims(pen, node_count, fd);
    float x[3 * 64], ang[3 * 64] = {0};  /* expand_angles fills ang[0 .. 3J) */
    for (int d = 0; d < D; d++) x[d] = particles[pidx(count, i, 0, d, D)];
    expand_angles(chain, node_count, pen, x, ang);
    return fitness_pen(chain, node_count, positions, ang, aw, dw, pen);
}

/* Node world positions (xyz) for nodes 1..J: out[3*(k-1)+c]. */
void orc_node_positions(const orc_node* chain, int node_count, const float* angles, float* out)
{
    float mats[64 * 16];
    orc_chain_matrices(chain, node_count, angles, mats);
    for (int k = 1; k < node_count; k++) {
        out[3 * (k - 1) + 0] = mats[16 * k + 3];
        out[3 * (k - 1) + 1] = mats[16 * k + 7];
        out[3 * (k - 1) + 2] = mats[16 * k + 11];
    }
}

/* checkDistance (src/Main.cpp:290-298): sum over effectors of Euclidean distance to target. */
float orc_residual(const orc_node* chain, int node_count, const float* angles)
{
    float mats[64 * 16];
    orc_chain_matrices(chain, node_count, angles, mats);
    float dist = 0.0f;
    for (int k = 1; k < node_count; k++) {
        if (chain[k].node_type != ORC_EFFECTOR) continue;
        float dx = chain[k].target_position[0] - mats[16 * k + 3];
        float dy = chain[k].target_position[1] - mats[16 * k + 7];
        float dz = chain[k].target_position[2] - mats[16 * k + 11];
        dist += sqrtf(dx * dx + dy * dy + dz * dz);
    }
    return dist;
}

/* ------------------------------------------------------------ PSO driver */

/* First index of the minimum, operator< (thrust::min_element semantics). */
static int64_t argmin_first(const float* v, int64_t n)
{
    int64_t best = 0;
    for (int64_t i = 1; i < n; i++)
        if (v[i] < v[best]) best = i;
    return best;
}

/* calculatePSO (src/kernel.cu:279-327); orc_calculate_pso: colliderCount = 0, _ex: any.
 * particles: [3][dof][size] SoA (position, velocity, localBest); bests[size];
 * randoms[size]; result[dof].  Returns 0. */
static int calculate_pso_pen(float* particles, const float* positions, float* bests, orc_rng* randoms,
                             int64_t size, const orc_node* chain, int node_count, float inertia, float local,
                             float global, int iterations, float angle_weight, float distance_weight,
                             float* result, const orc_extra* pen);

int orc_calculate_pso(float* particles, const float* positions, float* bests, orc_rng* randoms, int64_t size,
                      const orc_node* chain, int node_count, float inertia, float local, float global,
                      int iterations, float angle_weight, float distance_weight, float* result)
{
    return calculate_pso_pen(particles, positions, bests, randoms, size, chain, node_count, inertia, local, global,
                             iterations, angle_weight, distance_weight, result, NULL);
}

int orc_calculate_pso_ex(float* particles, const float* positions, float* bests, orc_rng* randoms, int64_t size,
                         const orc_node* chain, int node_count, float inertia, float local, float global,
                         int iterations, float angle_weight, float distance_weight, float* result,
                         float limit_weight, const float* soft_lo, const float* soft_hi, const void* colliders,
                         int collider_count)
{
    orc_extra pen = {limit_weight, soft_lo, soft_hi, colliders, collider_count, NULL};
    return calculate_pso_pen(particles, positions, bests, randoms, size, chain, node_count, inertia, local, global,
                             iterations, angle_weight, distance_weight, result, &pen);
}

static int calculate_pso_pen(float* particles, const float* positions, float* bests, orc_rng* randoms,
                             int64_t size, const orc_node* chain, int node_count, float inertia, float local,
                             float global, int iterations, float angle_weight, float distance_weight,
                             float* result, const orc_extra* pen)
{
    /* dof = the free dimensions (3 per node without an axis mask, the reference) */
    int fd[3 * 64];
    const int dof = free_dims(pen, node_count, fd);
    const int64_t n = size;

    /* initParticlesKernel (src/kernel.cu:223-266) */
    for (int64_t i = 0; i < n; i++) {
        for (int d = 0; d < dof; d++) {
            const int ci = fd[d] / 3 + 1;
            particles[pidx(n, i, 0, d, dof)] = chain[ci].rotation[fd[d] % 3];
        }
        for (int d = 0; d < dof; d++) {
            particles[pidx(n, i, 1, d, dof)] = orc_curand_uniform(&randoms[i]) * 2.0f - 1.0f;
            particles[pidx(n, i, 2, d, dof)] = particles[pidx(n, i, 0, d, dof)];
        }
    }
    /* initLocalBests */
    for (int64_t i = 0; i < n; i++)
        bests[i] = fitness_soa(chain, node_count, positions, particles, n, i, angle_weight, distance_weight, pen);

    int64_t g = argmin_first(bests, n);
    for (int d = 0; d < dof; d++) result[d] = particles[pidx(n, g, 2, d, dof)];
    float global_min = bests[g];

    for (int it = 0; it < iterations; it++) {
        /* simulateParticlesKernel (src/kernel.cu:153-189) */
        for (int64_t i = 0; i < n; i++) {
            for (int d = 0; d < dof; d++) {
                int64_t vi = pidx(n, i, 1, d, dof), xi = pidx(n, i, 0, d, dof), bi = pidx(n, i, 2, d, dof);
                float r1 = orc_curand_uniform(&randoms[i]);
                float r2 = orc_curand_uniform(&randoms[i]);
                float r3 = orc_curand_uniform(&randoms[i]);
                particles[vi] = inertia * r1 * particles[vi] + local * r2 * (particles[bi] - particles[xi]) +
                                global * r3 * (result[d] - particles[xi]);
                particles[xi] += particles[vi];
            }
            for (int d = 0; d < dof; d++) {
                const int k = fd[d] / 3 + 1, c = fd[d] % 3;
                int64_t xi = pidx(n, i, 0, d, dof);
                particles[xi] = clampf_ref(particles[xi], chain[k].min_rotation[c], chain[k].max_rotation[c]);
            }
        }
        /* updateLocalBests (src/kernel.cu:202-221) */
        for (int64_t i = 0; i < n; i++) {
            float f = fitness_soa(chain, node_count, positions, particles, n, i, angle_weight, distance_weight, pen);
            if (f < bests[i]) {
                bests[i] = f;
                for (int d = 0; d < dof; d++) particles[pidx(n, i, 2, d, dof)] = particles[pidx(n, i, 0, d, dof)];
            }
        }
        g = argmin_first(bests, n);
        float cur = bests[g];
        if (global_min > cur) {
            global_min = cur;
            for (int d = 0; d < dof; d++) result[d] = particles[pidx(n, g, 2, d, dof)];
        }
    }
    return 0;
}

/* ----------------------------------------------------- batch (CPU baseline)
 * B independent reference solves.  Swarm b uses `chain` with its effector
 * targets replaced by targets[b] ([B][E][3], effectors in node order) and, if
 * start_pose is non-NULL, its node rotations replaced by start_pose[b] ([B][D];
 * warm start + angle-term reference, as Node::ToCUDA does per frame).
 * rng: [B][P] states, persisting across calls.
 * Outputs: angles[B][D], fitness[B], residual[B] (residual may be NULL).
 * limit_weight/soft_lo/soft_hi: optional penalty extension (0/NULL = off).
 * colliders/collider_count: obj_t boxes of the collider term (0 = off).
 * Parallel over swarms with OpenMP (threads <= 0: runtime default). */
int orc_solve_batch_mask(const orc_node* chain, int node_count, const float* targets, const float* start_pose,
                         int64_t num_swarms, int particles_per_swarm, int iterations, float inertia, float local,
                         float global, float angle_weight, float distance_weight, const float* positions,
                         orc_rng* rng, float* out_angles, float* out_fitness, float* out_residual, int threads,
                         float limit_weight, const float* soft_lo, const float* soft_hi, const void* colliders,
                         int collider_count, const uint8_t* axis_mask);

int orc_solve_batch(const orc_node* chain, int node_count, const float* targets, const float* start_pose,
                    int64_t num_swarms, int particles_per_swarm, int iterations, float inertia, float local,
                    float global, float angle_weight, float distance_weight, const float* positions,
                    orc_rng* rng, float* out_angles, float* out_fitness, float* out_residual, int threads,
                    float limit_weight, const float* soft_lo, const float* soft_hi, const void* colliders,
                    int collider_count)
{
    return orc_solve_batch_mask(chain, node_count, targets, start_pose, num_swarms, particles_per_swarm, iterations,
                                inertia, local, global, angle_weight, distance_weight, positions, rng, out_angles,
                                out_fitness, out_residual, threads, limit_weight, soft_lo, soft_hi, colliders,
                                collider_count, NULL);
}

/* axis_mask: see orc_extra (NULL = the reference); start_pose [B][D], out_angles [B][D]
 * over the D free dimensions. */
int orc_solve_batch_mask(const orc_node* chain, int node_count, const float* targets, const float* start_pose,
                         int64_t num_swarms, int particles_per_swarm, int iterations, float inertia, float local,
                         float global, float angle_weight, float distance_weight, const float* positions,
                         orc_rng* rng, float* out_angles, float* out_fitness, float* out_residual, int threads,
                         float limit_weight, const float* soft_lo, const float* soft_hi, const void* colliders,
                         int collider_count, const uint8_t* axis_mask)
{
    const int64_t P = particles_per_swarm;
    orc_extra pen = {limit_weight, soft_lo, soft_hi, colliders, collider_count, axis_mask};
    const orc_extra* penp = &pen;
    if (node_count > 64 || node_count < 2) return 1;
    int fd[3 * 64];
    const int dof = free_dims(penp, node_count, fd);
    int num_eff = 0;
    for (int k = 1; k < node_count; k++) num_eff += chain[k].node_type == ORC_EFFECTOR;
    int err = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t b = 0; b < num_swarms; b++) {
        orc_node lc[64];
        float* parts = (float*)malloc(sizeof(float) * 3 * dof * P);
        float* bests = (float*)malloc(sizeof(float) * P);
        if (!parts || !bests) {
#pragma omp atomic write
            err = 2;
            free(parts);
            free(bests);
            continue;
        }
        memcpy(lc, chain, sizeof(orc_node) * node_count);
        if (start_pose)
            for (int d = 0; d < dof; d++) lc[fd[d] / 3 + 1].rotation[fd[d] % 3] = start_pose[b * dof + d];
        int e = 0;
        for (int k = 1; k < node_count; k++) {
            if (lc[k].node_type == ORC_EFFECTOR) {
                if (targets)
                    for (int c = 0; c < 3; c++) lc[k].target_position[c] = targets[(b * num_eff + e) * 3 + c];
                e++;
            }
        }
        float* res = out_angles + b * dof;
        calculate_pso_pen(parts, positions, bests, rng + b * P, P, lc, node_count, inertia, local, global,
                          iterations, angle_weight, distance_weight, res, penp);
        float gmin = bests[0];
        for (int64_t i = 1; i < P; i++)
            if (bests[i] < gmin) gmin = bests[i];
        out_fitness[b] = gmin;
        if (out_residual) {
            float full[3 * 64];
            expand_angles(lc, node_count, penp, res, full);
            out_residual[b] = orc_residual(lc, node_count, full);
        }
        free(parts);
        free(bests);
    }
    return err;
}
