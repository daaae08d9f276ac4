// ikpso_api.cpp -- the C ABI (include/ikpso.h): validation, chain parsing,
// solver handles, dispatch to the gfx950 kernels.
#include <hip/hip_runtime.h>

#include <math.h>

#include <cmath>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include <array>
#include <atomic>
#include <mutex>
#include <new>
#include <vector>

#include "ikpso.h"
#include "ikpso_kernels.h"

using namespace ikpso;

// csrc/_build/ikpso_build_id.cpp, written by the Makefile on every build
extern "C" const char ikpso_build_id_string[];

static_assert(sizeof(ikpso_node) == 88, "ikpso_node must match NodeCUDA (88 bytes)");
static_assert(sizeof(ikpso_rng_state) == 48, "ikpso_rng_state must match curandStateXORWOW (48 bytes)");
static_assert(sizeof(ikpso_pso_config) == 16, "PSOConfig is 16 bytes");
static_assert(sizeof(ikpso_fitness_config) == 12, "FitnessConfig is 12 bytes");
static_assert(sizeof(ikpso_collider) == 48, "obj_t is 48 bytes");

// Collider-term counters of an IKPSO_COLLIDE_STATS build (tools/collide_stats.py):
// one device block for the process, read and cleared by ikpso_debug_collide_stats.
unsigned long long* ikpso::collide_stats_buffer()
{
#if IKPSO_COLLIDE_STATS
    static unsigned long long* buf = nullptr;
    if (!buf && hipMalloc(&buf, kCsCount * sizeof(unsigned long long)) == hipSuccess)
        (void)hipMemset(buf, 0, kCsCount * sizeof(unsigned long long));
    return buf;
#else
    return nullptr;
#endif
}

#if IKPSO_COLLIDE_STATS
// [kCsCount] counters since the last reset (reset != 0 clears them after the read).
extern "C" int ikpso_debug_collide_stats(unsigned long long* out, int reset)
{
    unsigned long long* buf = ikpso::collide_stats_buffer();
    if (!buf) return (int)hipErrorMemoryAllocation;
    hipError_t e = hipMemcpy(out, buf, ikpso::kCsCount * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    if (e == hipSuccess && reset) e = hipMemset(buf, 0, ikpso::kCsCount * sizeof(unsigned long long));
    return (int)e;
}
#endif

namespace {

thread_local int g_last_hip_error = 0;
std::atomic<int64_t> g_coop_fallbacks{0};  // cooperative solves re-run on the streaming kernels

ikpso_status hip_status(hipError_t e)
{
    if (e == hipSuccess) return IKPSO_OK;
    g_last_hip_error = (int)e;
    return e == hipErrorOutOfMemory ? IKPSO_ERR_NO_MEMORY : IKPSO_ERR_HIP;
}

#define IKPSO_HIP(call)                                  \
    do {                                                 \
        hipError_t e_ = (call);                          \
        if (e_ != hipSuccess) return hip_status(e_);     \
    } while (0)

// ---- reference-order 4x4 host math for the origin transform M0 -----------
// M0 = I * T(position) * Rx * Ry * Rz (src/kernel.cu:36-38), computed with
// the reference's product order so the REFERENCE arithmetic mode reproduces
// it bit for bit.
struct M4 {
    float c[16];
};

M4 m4_create(float f)
{
    M4 m;
    for (float& x : m.c) x = 0.0f;
    for (int i = 0; i < 4; ++i) m.c[i + 4 * i] = f;
    return m;
}

M4 m4_mul(const M4& l, const M4& r)
{
#pragma clang fp contract(off)
    M4 o = m4_create(0.0f);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float s = 0.0f;
            for (int x = 0; x < 4; ++x) s += l.c[x + j * 4] * r.c[x * 4 + i];
            o.c[i + j * 4] = s;
        }
    return o;
}

// Correctly rounded fp32 sin/cos: what the device REFERENCE mode computes.
float sin_cr(float x) { return (float)sin((double)x); }
float cos_cr(float x) { return (float)cos((double)x); }

M4 origin_matrix(const ikpso_node& n)
{
    M4 m = m4_create(1.0f);
    M4 t = m4_create(1.0f);
    t.c[3] = n.position[0];
    t.c[7] = n.position[1];
    t.c[11] = n.position[2];
    m = m4_mul(m, t);
    const float a = n.rotation[0], b = n.rotation[1], c = n.rotation[2];
    M4 rx = m4_create(1.0f);
    rx.c[5] = cos_cr(a);
    rx.c[6] = -sin_cr(a);
    rx.c[9] = sin_cr(a);
    rx.c[10] = cos_cr(a);
    m = m4_mul(m, rx);
    M4 ry = m4_create(1.0f);
    ry.c[0] = cos_cr(b);
    ry.c[2] = sin_cr(b);
    ry.c[8] = -sin_cr(b);
    ry.c[10] = cos_cr(b);
    m = m4_mul(m, ry);
    M4 rz = m4_create(1.0f);
    rz.c[0] = cos_cr(c);
    rz.c[1] = -sin_cr(c);
    rz.c[4] = sin_cr(c);
    rz.c[5] = cos_cr(c);
    return m4_mul(m, rz);
}

uint32_t as_bits(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

// Copy `bytes` from host, managed or device memory into host memory.
// Pageable host memory (what a caller's plain arrays are; the Python mirror's
// numpy tables) is copied on the CPU: nothing on the GPU can be writing it, and
// the per-frame node table then costs no device round trip.  Pinned host,
// device and managed memory go through hipMemcpy, which orders the read after
// the caller's queued GPU work (an async copy that fills a pinned buffer, or a
// kernel writing the managed node table).
ikpso_status fetch_any(void* dst, const void* src, size_t bytes)
{
    if (bytes == 0) return IKPSO_OK;
    // hipPointerGetAttributes reports an unregistered host pointer as an error and
    // records it as the thread's last error: clear it (the entry points have taken
    // any error the caller's own earlier work left, take_pending_error)
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, src);
    if (e != hipSuccess) (void)hipGetLastError();
    if (e != hipSuccess || a.type == hipMemoryTypeUnregistered) {
        memcpy(dst, src, bytes);
        return IKPSO_OK;
    }
    IKPSO_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
    return IKPSO_OK;
}

// An error the caller's earlier HIP work left pending (not yet read by
// hipGetLastError) is reported up front by the next entry point that runs HIP
// work (calculate_pso, solver_create, solve_batch), which then leaves every buffer
// and the solver state untouched.  The reference's calculatePSO also returns such
// an error, from its first cudaGetLastError check (src/kernel.cu:293-295), but only
// after its init kernels have already rewritten particles, bests and randoms.
// Taking it here also keeps it from being mistaken for a launch failure of this
// call (the launches are checked with hipGetLastError) and from being cleared by
// fetch_any / is_device_memory, which clear the errors their own lookups cause.
hipError_t take_pending_error() { return hipGetLastError(); }

struct Extras {
    const float* positions = nullptr;  // host copy, [4J]
    float limit_weight = 0.0f;
    const float* soft_lo = nullptr;    // host copies, [D]
    const float* soft_hi = nullptr;
    const ikpso_collider* colliders = nullptr;  // host copy, [collider_count]
    int collider_count = 0;
    // IKPSO_FLAG_POSREF_NODE_SLOT: positions[] is [4*(J+2)] and node k's
    // reference position is read from slot k+1 (where FillPositions wrote it)
    bool posref_node_slot = false;
    const uint8_t* axis_mask = nullptr;  // host copy, [J + 1] (entry 0 ignored), or null
};

// ---- the folded serial chain (TopoDH), fp64 host algebra ------------------
struct D3 {
    double m[3][3];
};

D3 d3_eye()
{
    D3 r{};
    for (int i = 0; i < 3; ++i) r.m[i][i] = 1.0;
    return r;
}

D3 d3_mul(const D3& a, const D3& b)
{
    D3 r{};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            for (int x = 0; x < 3; ++x) r.m[i][j] += a.m[i][x] * b.m[x][j];
    return r;
}

// Rx / Ry / Rz of the reference (src/matrix_operations.cuh:136-161)
D3 d3_rot(int axis, double t)
{
    D3 r = d3_eye();
    const double c = cos(t), s = sin(t);
    const int i = (axis + 1) % 3, j = (axis + 2) % 3;  // x: (y, z); y: (z, x); z: (x, y)
    r.m[i][i] = c;
    r.m[i][j] = -s;
    r.m[j][i] = s;
    r.m[j][j] = c;
    return r;
}

// Q_c with Q_c Rz(t) Q_c^T = R_c(t): the cyclic permutation taking z to axis c.
D3 d3_q(int c)
{
    D3 r{};
    for (int i = 0; i < 3; ++i) r.m[(i + c + 1) % 3][i] = 1.0;  // Q e_i = e_{(i + c + 1) % 3}
    return r;
}

D3 d3_t(const D3& a)
{
    D3 r{};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[j][i];
    return r;
}

// Device record of one obj_t collider (ikpso_collide.h): the inverse
// quaternion is quatInvert2's (same fp32 operations as the device would do)
// and the radius bounds every support point of the box.
CollRec collider_record(const ikpso_collider& c)
{
    CollRec r{};
    r.px = c.pos[0];
    r.py = c.pos[1];
    r.pz = c.pos[2];
    r.qx = c.quat[0];
    r.qy = c.quat[1];
    r.qz = c.quat[2];
    r.qw = c.quat[3];
    float qi[4];
    quat_inverse(c.quat, qi);
    r.ix = qi[0];
    r.iy = qi[1];
    r.iz = qi[2];
    r.iw = qi[3];
    r.sx = c.x;
    r.sy = c.y;
    r.sz = c.z;
    r.radius = sphere_radius(fabsf(c.x), fabsf(c.y), fabsf(c.z), quat_gain(c.quat[0], c.quat[1], c.quat[2], c.quat[3]));
    return r;
}

// The collider as an oriented box for the FAST separating-axis test (kFastSat): the
// columns of the linear map quatRotVec(., q) (src/kernel.cu:1012-1037) -- the box's
// axes -- computed in fp64, the half extents and the centre: box[0..8] = axes (axis
// c at box[3c..3c+2], normalised), box[9..11] = |x, y, z| / 2 times the columns'
// lengths, box[12..14] = centre.  A quaternion a little off unit length (the
// reference's initColliders box 1 has |q|^2 = 1.0001) makes the map a rotation scaled
// and skewed by ~|q|^2 - 1: below 1e-3 that moves the box's faces by less than GJK's
// own ~3.5e-4 tolerance band; beyond it (false) the FAST builds test it by GJK.
bool collider_box(const ikpso_collider& c, float* box)
{
    const double x = c.quat[0], y = c.quat[1], z = c.quat[2], w = c.quat[3];
    double m[3][3];  // m[row][col]: quatRotVec(e_col)
    for (int col = 0; col < 3; ++col) {
        const double v[3] = {col == 0 ? 1.0 : 0.0, col == 1 ? 1.0 : 0.0, col == 2 ? 1.0 : 0.0};
        const double c1x = y * v[2] - z * v[1] + w * v[0], c1y = z * v[0] - x * v[2] + w * v[1],
                     c1z = x * v[1] - y * v[0] + w * v[2];
        const double c2x = y * c1z - z * c1y, c2y = z * c1x - x * c1z, c2z = x * c1y - y * c1x;
        m[0][col] = v[0] + 2.0 * c2x;
        m[1][col] = v[1] + 2.0 * c2y;
        m[2][col] = v[2] + 2.0 * c2z;
    }
    bool ortho = true;
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            const double d = m[0][a] * m[0][b] + m[1][a] * m[1][b] + m[2][a] * m[2][b];
            ortho = ortho && fabs(d - (a == b ? 1.0 : 0.0)) <= 1e-3;
        }
    const double half[3] = {0.5 * fabs((double)c.x), 0.5 * fabs((double)c.y), 0.5 * fabs((double)c.z)};
    for (int col = 0; col < 3; ++col) {
        const double n = sqrt(m[0][col] * m[0][col] + m[1][col] * m[1][col] + m[2][col] * m[2][col]);
        ortho = ortho && n > 0.0;
        for (int row = 0; row < 3; ++row) box[3 * col + row] = (float)(n > 0.0 ? m[row][col] / n : 0.0);
        box[9 + col] = (float)(half[col] * n);
    }
    box[12] = c.pos[0];
    box[13] = c.pos[1];
    box[14] = c.pos[2];
    box[15] = 0.0f;
    return ortho;
}

ikpso_status parse_chain(const std::vector<ikpso_node>& nodes, const ikpso_pso_config& pso,
                         const ikpso_fitness_config& fit, const Extras& ex, ChainHost& ch)
{
    const int n = (int)nodes.size();
    if (n < 2 || n - 1 > kMaxJoints) return IKPSO_ERR_INVALID_ARG;
    const int J = n - 1;
    ch = ChainHost{};
    ch.J = J;
    ch.parent.assign(J + 1, -1);
    ch.eff_slot.assign(J + 1, -1);
    ch.len.assign(J + 1, 0.0f);
    ch.eff_w.assign(J + 1, 0.0f);
    ch.lo.assign(3 * J, 0.0f);
    ch.hi.assign(3 * J, 0.0f);
    ch.rest.assign(3 * J, 0.0f);
    ch.tgt0.assign(3 * J, 0.0f);
    int E = 0;
    bool ref7 = (J == 7), serial = true;
    uint64_t eff_mask = 0;
    static const int kRef7[8] = {-1, 0, 1, 2, 3, 4, 4, 4};
    for (int k = 1; k <= J; ++k) {
        const ikpso_node& nd = nodes[k];
        if (nd.parent_index < 0 || nd.parent_index >= k) return IKPSO_ERR_INVALID_ARG;
        ch.parent[k] = nd.parent_index;
        ch.len[k] = nd.length;
        serial = serial && nd.parent_index == k - 1;
        if (J == 7) ref7 = ref7 && nd.parent_index == kRef7[k];
        for (int c = 0; c < 3; ++c) {
            ch.lo[3 * (k - 1) + c] = nd.min_rotation[c];
            ch.hi[3 * (k - 1) + c] = nd.max_rotation[c];
            ch.rest[3 * (k - 1) + c] = nd.rotation[c];
        }
        if (nd.node_type == IKPSO_NODE_EFFECTOR) {
            eff_mask |= 1ull << k;
            ch.eff_slot[k] = E++;
            ch.eff_w[k] = nd.effector_weight;
            for (int c = 0; c < 3; ++c) ch.tgt0[3 * (k - 1) + c] = nd.target_position[c];
        }
    }
    ch.E = E;
    // joint-axis mask: bit d = 3(k-1)+c of free_mask when Euler angle c of node k is free
    ch.free_mask = 0;
    for (int k = 1; k <= J; ++k)
        for (int c = 0; c < 3; ++c) {
            const int d = 3 * (k - 1) + c;
            if (d >= 64) break;  // > 21 joints: no compiled kernel (rejected below)
            if (!ex.axis_mask || ((ex.axis_mask[k] >> c) & 1)) ch.free_mask |= 1ull << d;
        }
    for (int k = 1; k <= J && ex.axis_mask; ++k)
        if (ex.axis_mask[k] > 7) return IKPSO_ERR_INVALID_ARG;
    ch.dfree = __builtin_popcountll(ch.free_mask);
    ch.masked = 3 * J <= 64 && ch.dfree != 3 * J;
    if (ch.dfree == 0) return IKPSO_ERR_INVALID_ARG;  // nothing to optimise
    ch.uniform_bounds = true;
    for (int d = 0; d < 3 * J && ch.uniform_bounds; ++d)
        ch.uniform_bounds = ch.uniform_bounds && as_bits(ch.lo[d]) == as_bits(ch.lo[0]) &&
                            as_bits(ch.hi[d]) == as_bits(ch.hi[0]);
    // [0, 2pi] limits are [0, 1] in revolutions (ChainConsts::rlo / rhi, the same fp32 products)
    {
        volatile float inv = 0.159154943091895336f;  // (no contraction or constant folding differences)
        const float rlo = ch.lo[0] * inv, rhi = ch.hi[0] * inv;
        ch.unit_rev_bounds = ch.uniform_bounds && rlo == 0.0f && rhi == 1.0f;
        ch.ordered_bounds = ch.uniform_bounds && std::isfinite(ch.lo[0]) && std::isfinite(ch.hi[0]) &&
                            ch.lo[0] <= ch.hi[0];
    }
    ref7 = ref7 && eff_mask == 0xE0ull;                // effectors = nodes 5, 6, 7
    serial = serial && eff_mask == (1ull << J);        // single tip effector
    ch.topo = ref7 ? TopoKind::Ref7 : (serial ? TopoKind::SerialTip : TopoKind::Generic);
    const M4 m0 = origin_matrix(nodes[0]);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) ch.m0[4 * r + c] = m0.c[4 * r + c];
    ch.w = pso.inertia;
    ch.c1 = pso.local;
    ch.c2 = pso.global;
    // fitConfig.{angle,distance}Weight / (DEGREES_OF_FREEDOM / 3) (src/kernel.cu:150)
    ch.aw_j = fit.angle_weight / (float)J;
    ch.dw_j = fit.distance_weight / (float)J;
    ch.use_posref = fit.distance_weight != 0.0f;
    ch.lim_w = ex.limit_weight;
    ch.use_penalty = ex.limit_weight != 0.0f && ex.soft_lo && ex.soft_hi;
    // aux = [posref 4J | soft_lo 3J | soft_hi 3J | pad to 16 floats | collider records | near limits |
    //        collider boxes], the colliders being those within the arm's reach (below)
    //
    // near_collider's limit for node k and collider c (ikpso_collide.h): one sphere around
    // the node's link box and node box, centred at the link's midpoint, that any box pair
    // node_collides would test lies within.  Every node position is within
    // |origin| + sum |len| of the frame's origin (a bound on the exact test's |centre|_1
    // margin term through |a|_1 <= sqrt(3) |a|).
    //
    // Host-side pruning: every node (and link midpoint) lies within the arm's length sum
    // sum_k |len_k| of the origin's position, so a collider farther from it than that plus
    // near_collider's limit for every node can never pass the inline sphere test, let
    // alone the exact one (the margin covers the fp32 FK's rounding, ~1e-6 of the reach):
    // it can never contribute to any fitness, and is left out.  With none left the chain
    // is solved without the term, by the plain kernels -- bit-identical answers in
    // REFERENCE arithmetic (the same reference operation order), and in FAST the plain
    // kernels' own arithmetic.  IKPSO_KEEP_FAR_COLLIDERS=1 keeps every collider (to time
    // the collider kernels with nothing near).
    double reach = sqrt((double)ch.m0[3] * ch.m0[3] + (double)ch.m0[7] * ch.m0[7] + (double)ch.m0[11] * ch.m0[11]);
    double arm = 0.0;
    for (int k = 1; k <= J; ++k) arm += fabs((double)ch.len[k]);
    reach = (reach + arm) * 1.001;
    const double gb = (double)kGainBound, lw = (double)kGizmo * 0.25;
    const double rn = 0.5 * sqrt(3.0) * (double)kGizmo * gb;
    const int nin = ex.collider_count;
    std::vector<CollRec> recs(nin);
    std::vector<float> lims((size_t)nin * J);
    std::vector<int> kept;
    const char* keep = getenv("IKPSO_KEEP_FAR_COLLIDERS");
    const bool keep_all = keep && keep[0] == '1';
    for (int i = 0; i < nin; ++i) {
        const CollRec r = recs[i] = collider_record(ex.colliders[i]);
        if (!std::isfinite(r.radius) || !std::isfinite(r.px) || !std::isfinite(r.py) || !std::isfinite(r.pz))
            return IKPSO_ERR_INVALID_ARG;
        const double c1 = fabs((double)r.px) + fabs((double)r.py) + fabs((double)r.pz);
        const double dx = (double)r.px - ch.m0[3], dy = (double)r.py - ch.m0[7], dz = (double)r.pz - ch.m0[11];
        const double dist = sqrt(dx * dx + dy * dy + dz * dz);
        const double margin = 1e-3 + 1e-4 * (arm + dist + c1);
        bool reachable = false;
        for (int k = 1; k <= J; ++k) {
            const double len = fabs((double)ch.len[k]);
            const double rl = 0.5 * sqrt(len * len + 2.0 * lw * lw) * gb;
            const double rk = std::max(rl, 0.5 * len * 1.00001 + rn);
            const double reach_kc = rk + (double)r.radius;
            const double lim = (reach_kc + 1e-3 + 1e-4 * (sqrt(3.0) * reach + c1 + reach_kc)) * 1.0001;
            if (!std::isfinite(lim)) return IKPSO_ERR_INVALID_ARG;
            lims[(size_t)i * J + (k - 1)] = (float)(lim * lim);
            reachable = reachable || dist - arm <= sqrt((double)lims[(size_t)i * J + (k - 1)]) + margin;
        }
        if (reachable || keep_all) kept.push_back(i);
    }
    ch.colliders_dropped = nin - (int)kept.size();
    ch.num_coll = (int)kept.size();
    ch.coll_off = ((size_t)10 * J + 15) & ~size_t(15);
    ch.coll_lim_off = ch.coll_off + (size_t)16 * ch.num_coll;
    ch.coll_box_off = (ch.coll_lim_off + (size_t)J * ch.num_coll + 15) & ~size_t(15);
    ch.aux.assign(ch.coll_box_off + (size_t)16 * ch.num_coll, 0.0f);
    for (int j = 0; j < ch.num_coll; ++j) {
        const int i = kept[j];
        memcpy(ch.aux.data() + ch.coll_off + 16 * (size_t)j, &recs[i], sizeof(CollRec));
        ch.coll_obb = ch.coll_obb && collider_box(ex.colliders[i], ch.aux.data() + ch.coll_box_off + 16 * (size_t)j);
        for (int k = 1; k <= J; ++k)
            ch.aux[ch.coll_lim_off + (size_t)(k - 1) * ch.num_coll + j] = lims[(size_t)i * J + (k - 1)];
    }
    if (ch.use_posref && ex.positions)
        for (int i = 0; i < 4 * J; ++i) ch.aux[i] = ex.positions[i + (ex.posref_node_slot ? 8 : 0)];
    if (ch.use_penalty)  // soft limits are given per free dimension; a locked angle adds max(-inf, 0)^2 = 0
        for (int d = 0, r = 0; d < 3 * J; ++d) {
            const bool fr = d < 64 && ((ch.free_mask >> d) & 1);
            ch.aux[4 * J + d] = fr ? ex.soft_lo[r] : -INFINITY;
            ch.aux[7 * J + d] = fr ? ex.soft_hi[r] : INFINITY;
            r += fr;
        }
    // the transcendental unit's range (kHwTrigMaxAbs): every evaluated angle is
    // clamped to [lo, hi] after the first update, the warm start is the rest pose
    for (int d = 0; d < 3 * J && d < 64; ++d)
        if ((ch.free_mask >> d) & 1)
            ch.poly_trig = ch.poly_trig || !(fabsf(ch.lo[d]) <= kHwTrigMaxAbs) || !(fabsf(ch.hi[d]) <= kHwTrigMaxAbs) ||
                           !(fabsf(ch.rest[d]) <= kHwTrigMaxAbs);
    // symmetric soft limits within one revolution of every clamp bound (kTermSymPenalty): checked in the
    // kernels' revolution units, where the overshoot |x| - h of a clamped angle is <= 1
    if (ch.use_penalty && ch.uniform_bounds) {
        volatile float inv = 0.159154943091895336f;
        const float rmax = fmaxf(fabsf(ch.lo[0] * inv), fabsf(ch.hi[0] * inv));
        ch.sym_penalty = true;
        for (int d = 0; d < 3 * J; ++d) {
            const float slo = ch.aux[4 * J + d], shi = ch.aux[7 * J + d];
            ch.sym_penalty = ch.sym_penalty && as_bits(slo) == (as_bits(shi) ^ 0x80000000u) && shi >= 0.0f &&
                             rmax - shi * inv <= 1.0f;
        }
    }
    if (!chain_supported(ch)) return IKPSO_ERR_UNSUPPORTED;
    return IKPSO_OK;
}

// Number of compiled TopoDH instantiations (ikpso_inst_dh_*.hip).
constexpr int kDHMin = 3, kDHMax = 12;

// The folded form of a masked serial chain with a tip effector (TopoDH, FAST
// kernels): every free Euler axis becomes one joint W_j = W_{j-1} C_j Rz(t_j),
// q_j = q_{j-1} + W_j s_j (see TopoDH).  The constants are products of the
// locked rotations (at their rest angles), the axis permutations Q_c, the
// origin transform and the link translations, multiplied out in fp64 and
// rounded once.  False when the chain does not fold (tree, several effectors,
// distance or collider term, no compiled width).
bool build_dh(const std::vector<ikpso_node>& nodes, const ChainHost& eu, const Extras& ex, ChainHost& dh)
{
    const int J = eu.J, N = eu.dfree;
    if (eu.topo != TopoKind::SerialTip || eu.use_posref || eu.num_coll > 0 || !eu.masked || eu.poly_trig) return false;
    if (N < kDHMin || N > kDHMax) return false;
    const ikpso_node& o = nodes[0];
    D3 g = d3_mul(d3_mul(d3_rot(0, o.rotation[0]), d3_rot(1, o.rotation[1])), d3_rot(2, o.rotation[2]));
    double sc[3] = {o.position[0], o.position[1], o.position[2]};  // offset in the current joint frame
    std::vector<D3> C;
    std::vector<std::array<double, 3>> S;
    std::array<double, 3> q0{};
    for (int k = 1; k <= J; ++k) {
        for (int c = 0; c < 3; ++c) {
            const int d = 3 * (k - 1) + c;
            if ((eu.free_mask >> d) & 1) {
                if (C.empty())
                    q0 = {sc[0], sc[1], sc[2]};
                else
                    S.back() = {sc[0], sc[1], sc[2]};
                C.push_back(d3_mul(g, d3_q(c)));
                S.push_back({0.0, 0.0, 0.0});
                g = d3_t(d3_q(c));
                sc[0] = sc[1] = sc[2] = 0.0;
            } else {
                g = d3_mul(g, d3_rot(c, nodes[k].rotation[c]));
            }
        }
        const double len = nodes[k].length;  // T(len, 0, 0) after the node's rotation
        for (int r = 0; r < 3; ++r) sc[r] += len * g.m[r][0];
    }
    S.back() = {sc[0], sc[1], sc[2]};
    dh = ChainHost{};
    dh.J = N;
    dh.E = 1;
    dh.topo = TopoKind::DH;
    dh.parent.assign(N + 1, -1);
    dh.eff_slot.assign(N + 1, -1);
    dh.len.assign(N + 1, 0.0f);
    dh.eff_w.assign(N + 1, 0.0f);
    dh.lo.assign(3 * N, 0.0f);
    dh.hi.assign(3 * N, 0.0f);
    dh.rest.assign(3 * N, 0.0f);
    dh.tgt0.assign(3 * N, 0.0f);
    for (int k = 1; k <= N; ++k) dh.parent[k] = k - 1;
    dh.eff_slot[N] = 0;
    dh.eff_w[N] = eu.eff_w[J];
    for (int c = 0; c < 3; ++c) dh.tgt0[3 * (N - 1) + c] = eu.tgt0[3 * (J - 1) + c];
    for (int d = 0, r = 0; d < 3 * J; ++d)
        if ((eu.free_mask >> d) & 1) {
            dh.lo[r] = eu.lo[d];
            dh.hi[r] = eu.hi[d];
            dh.rest[r] = eu.rest[d];
            ++r;
        }
    dh.uniform_bounds = true;
    for (int d = 0; d < N; ++d)
        dh.uniform_bounds = dh.uniform_bounds && as_bits(dh.lo[d]) == as_bits(dh.lo[0]) &&
                            as_bits(dh.hi[d]) == as_bits(dh.hi[0]);
    dh.w = eu.w;
    dh.c1 = eu.c1;
    dh.c2 = eu.c2;
    dh.aw_j = eu.aw_j;  // angleWeight / node count of the chain, as calculateDistance
    dh.dw_j = 0.0f;
    dh.use_posref = false;
    dh.lim_w = eu.lim_w;
    dh.use_penalty = eu.use_penalty;
    dh.coll_off = ((size_t)10 * N + 15) & ~size_t(15);
    dh.dh_off = dh.coll_off;
    dh.aux.assign(dh.dh_off + 12 * (size_t)N + 4, 0.0f);
    if (dh.use_penalty)
        for (int d = 0, r = 0; d < 3 * J; ++d)
            if ((eu.free_mask >> d) & 1) {
                dh.aux[4 * N + r] = ex.soft_lo[r];
                dh.aux[7 * N + r] = ex.soft_hi[r];
                ++r;
            }
    dh.free_mask = (1ull << N) - 1;
    dh.dfree = N;
    dh.masked = false;
    float* dc = dh.aux.data() + dh.dh_off;
    for (int j = 0; j < N; ++j) {
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) dc[12 * j + 3 * r + c] = (float)C[j].m[r][c];
        for (int r = 0; r < 3; ++r) dc[12 * j + 9 + r] = (float)S[j][r];
    }
    for (int r = 0; r < 3; ++r) dc[12 * N + r] = (float)q0[r];
    return chain_supported(dh);
}

// Device scratch of the reference-compatible path (result staging, aux terms,
// streaming workspace).  The entry point holds g_scratch_mu for its whole call.
std::mutex g_scratch_mu;
float* g_scratch = nullptr;
size_t g_scratch_bytes = 0;

// What the per-frame call keeps between frames (under g_scratch_mu), so that a
// frame's device work is the solve kernel alone (round 4: the aux upload, the
// generator snapshot copy, the slot clear and two small D2H copies were 4 extra
// dependent operations of ~20 us around a 57 us kernel, profiles/r04/frame_*):
//  * aux: the last uploaded aux block and where it lies; a frame re-uploads only
//    when its content or place changed (the scene's bounds do not, per frame);
//  * slots: the cooperative slot region left by the last frame (CoopSlotState);
//  * pinned: [error flag | answer], written by the kernels themselves (coherent
//    pinned memory, read after the call's one synchronisation).
// A cooperative workspace's slot region between launches: [at, at + bytes)
// holds only zeros or granules tagged below `next`, so a launch there numbers
// its exchanges from `next` (SwarmIO::coop_tag0) instead of clearing the slots.
struct CoopSlotState {
    char* at = nullptr;
    size_t bytes = 0;
    uint32_t next = 0;
    void invalidate() { bytes = 0; }  // something else was written over the region
    // `exchanges`: an upper bound on the exchanges one group of the launch runs.
    hipError_t begin(SwarmIO& io, char* ws, size_t zero, uint64_t exchanges, hipStream_t s)
    {
        if (at != ws || zero > bytes || exchanges >= 0x7FFFFFFFull || (uint64_t)next + exchanges + 1 >= 0xFFFFFFFFull) {
            const hipError_t e = hipMemsetAsync(ws, 0, zero, s);
            if (e != hipSuccess) return e;
            next = 0;
        }
        io.coop_tag0 = next;
        next = exchanges >= 0x7FFFFFFFull ? 0xFFFFFFFFu : next + (uint32_t)exchanges + 1;  // (cleared next time)
        at = ws;
        bytes = zero;  // what lies past it (the snapshot, the fallback's workspace) is not known clean
        return hipSuccess;
    }
};

struct CompatFrameCache {
    const float* aux_at = nullptr;
    std::vector<float> aux;
    CoopSlotState slots;
    int32_t* pinned = nullptr;      // host address
    int32_t* pinned_dev = nullptr;  // its device address
};
CompatFrameCache g_frame;
constexpr size_t kFramePinnedWords = 64 + 3 * kMaxJoints;  // the flag, then the answer at word 64

ikpso_status scratch(size_t bytes, float** out)
{
    if (g_scratch_bytes < bytes) {
        if (g_scratch) (void)hipFree(g_scratch);
        g_scratch = nullptr;
        g_scratch_bytes = 0;
        g_frame.aux_at = nullptr;  // nothing of the old block is known to survive
        g_frame.slots.invalidate();
        IKPSO_HIP(hipMalloc(&g_scratch, bytes));
        g_scratch_bytes = bytes;
    }
    *out = g_scratch;
    return IKPSO_OK;
}

// True when `p` is memory of the current device (a kernel writes it directly;
// anything else -- pageable, pinned or managed host memory, another GPU's memory --
// gets the answer through the pinned block and a copy).
bool is_device_memory(const void* p)
{
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) (void)hipGetLastError();  // our own lookup's error (see fetch_any)
    int cur = -1;
    return e == hipSuccess && a.type == hipMemoryTypeDevice && hipGetDevice(&cur) == hipSuccess && a.device == cur;
}

// Carve 256-byte aligned arrays out of one allocation.
struct Carver {
    char* base;
    size_t off = 0;
    template <class T>
    T* take(size_t n)
    {
        off = (off + 255) & ~size_t(255);
        T* p = reinterpret_cast<T*>(base + off);
        off += n * sizeof(T);
        return p;
    }
};

// Streaming workspace layout (see StreamIO); state/pbf carved only when not
// supplied by the caller.
void carve_stream(StreamIO& io, void* ws, int64_t B, int P, int D, bool own_state)
{
    Carver cv{static_cast<char*>(ws)};
    const int C = (P + kStreamChunk - 1) / kStreamChunk;
    if (own_state) {
        io.state = cv.take<float>((size_t)B * 3 * D * P);
        io.pbf = cv.take<float>((size_t)B * P);
    }
    io.rng = cv.take<uint32_t>((size_t)6 * B * P);
    io.pkey = cv.take<uint32_t>((size_t)2 * B * C);
    io.pidx = cv.take<int32_t>((size_t)2 * B * C);
    io.pvec = cv.take<float>((size_t)2 * B * C * D);
    io.gkey = cv.take<uint32_t>((size_t)2 * B);
    io.gidx = cv.take<int32_t>((size_t)2 * B);
    io.gvec = cv.take<float>((size_t)2 * B * D);
    io.num_swarms = B;
    io.P = P;
    io.C = C;
}

int env_kernel()
{
    const char* e = getenv("IKPSO_KERNEL");
    if (!e) return IKPSO_KERNEL_AUTO;
    if (strcmp(e, "resident") == 0) return IKPSO_KERNEL_RESIDENT;
    if (strcmp(e, "streaming") == 0) return IKPSO_KERNEL_STREAMING;
    if (strcmp(e, "coop") == 0) return IKPSO_KERNEL_COOP;
    return IKPSO_KERNEL_AUTO;
}

// Cooperative launch plan for B swarms of P particles: chunk size (the
// throughput block, or with `latency` the 256-lane block when every swarm then
// still gets its own CUs), G chunks per swarm, NG concurrent groups (a
// multiple of 8 for the XCD-aware membership, kCoopBlocksPerCU workgroups per CU, at most
// ceil8(B)).  False if infeasible.
// *linear: a latency group wider than an XCD (G > CUs / 8: the visualiser's N =
// 16384 is 64 chunks) spans XCDs with linear membership (group = workgroup / G,
// NG = CUs / G, not a multiple of 8); its hand-offs cross XCDs (agent-scope
// granules are coherent there, MI355X_MICROARCH: +0.1-0.3 us per hop).
bool coop_plan(const ChainHost& ch, int mode, int P, int64_t B, bool latency, int* G, int* NG, int* block,
               bool* linear = nullptr)
{
    CoopGeometry geo;
    if (!coop_geometry(ch, mode, &geo)) return false;
    int T = geo.threads;
    if (linear) *linear = false;
    if (latency && geo.latency_variant) {
        const int gl = (P + kCoopLatencyThreads - 1) / kCoopLatencyThreads;
        if (gl <= 64 && B * gl <= (int64_t)geo.cus && ((geo.cus / gl) & ~7) >= 8) T = kCoopLatencyThreads;
        if (linear && T != kCoopLatencyThreads && gl <= 64 && B * gl <= (int64_t)geo.cus && coop_latency_split(ch)) {
            *G = gl;
            *NG = (int)std::min<int64_t>(B, geo.cus / gl);
            *block = kCoopLatencyThreads;
            *linear = true;
            return true;
        }
    }
    const int g = (P + T - 1) / T;
    int ng = (geo.cus * geo.blocks_per_cu / g) & ~7;
    if (g > 64 || ng < 8) return false;
    const int64_t want = ((B + 7) / 8) * 8;
    if (want < ng) ng = (int)want;
    *G = g;
    *NG = ng;
    *block = T;
    return true;
}

// AUTO for a swarm that fits one workgroup: the latency variant of the
// cooperative kernel when every swarm gets its own CUs (a few swarms: more
// CUs per swarm), else the resident kernel.
bool prefer_latency_coop(const ChainHost& ch, int mode, int P, int64_t B)
{
    int G, NG, T;
    return coop_plan(ch, mode, P, B, true, &G, &NG, &T) && T == kCoopLatencyThreads;
}

// Bound on a cooperative group wait (IKPSO_COOP_SPIN_LIMIT: debug knob; 0
// forces the give-up path so the fallback can be tested).
uint32_t coop_spin_limit()
{
    // only an explicit decimal number overrides the default: an empty or
    // malformed value (which strtoul would read as 0, the give-up path) is ignored
    const char* e = getenv("IKPSO_COOP_SPIN_LIMIT");
    if (!e || !*e) return kCoopSpinLimit;
    char* end = nullptr;
    const unsigned long v = strtoul(e, &end, 10);
    if (end == e || *end != '\0' || v > 0xFFFFFFFFul) return kCoopSpinLimit;
    return (uint32_t)v;
}

// Point the coop fields of `io` into workspace `ws` (coop_workspace_bytes) and
// clear the error flag and the slots (unless !clear: the caller numbers the
// exchanges past the tags the slots hold, io.coop_tag0).  *zero_bytes: the
// extent of the flag + slots from `ws`.
hipError_t carve_coop(SwarmIO& io, void* ws, int G, int NG, int block, int D, hipStream_t s, bool linear = false,
                      bool clear = true, size_t* zero_bytes = nullptr)
{
    io.coop_tag0 = 0;
    io.coop_spin_limit = coop_spin_limit();
    io.coop_linear = linear ? 1 : 0;
    Carver cv{static_cast<char*>(ws)};
    io.coop_error = cv.take<int32_t>(1);
    io.coop_slots = cv.take<unsigned long long>((size_t)NG * 2 * G * kCoopSlot(D));
    io.coop_timing = IKPSO_COOP_TIMING ? cv.take<unsigned long long>((size_t)NG * G * 8) : nullptr;
    io.coop_g = G;
    io.coop_ng = NG;
    io.coop_block = block;
    // the error flag and every granule's tag start at 0 (tags are exchange numbers + 1)
    const size_t zero = reinterpret_cast<char*>(io.coop_slots + (size_t)NG * 2 * G * kCoopSlot(D)) -
                        static_cast<char*>(ws);
    if (zero_bytes) *zero_bytes = zero;
    if (IKPSO_COOP_TIMING) {
        const hipError_t e = hipMemsetAsync(io.coop_timing, 0, (size_t)NG * G * 64, s);
        if (e != hipSuccess) return e;
    }
    return clear ? hipMemsetAsync(ws, 0, zero, s) : hipSuccess;
}

// Resolve the kernel family for a chain and swarm size; -1 if impossible.
int pick_kernel(const ChainHost& ch, int mode, int P, int requested)
{
    const bool fits = P <= resident_max_threads(ch);
    int G, NG, T;
    const bool coop = coop_plan(ch, mode, P, 1, false, &G, &NG, &T);
    if (requested == IKPSO_KERNEL_RESIDENT) return fits ? IKPSO_KERNEL_RESIDENT : -1;
    if (requested == IKPSO_KERNEL_STREAMING) return IKPSO_KERNEL_STREAMING;
    if (requested == IKPSO_KERNEL_COOP) return coop ? IKPSO_KERNEL_COOP : -1;
    return fits ? IKPSO_KERNEL_RESIDENT : (coop ? IKPSO_KERNEL_COOP : IKPSO_KERNEL_STREAMING);
}

}  // namespace

struct ikpso_solver {
    ChainHost chain;       // the node table as given (Euler form, with its axis mask)
    float* aux = nullptr;  // device copy of chain.aux
    // The folded form (TopoDH) a FAST solver of a masked serial chain solves with;
    // evaluate and REFERENCE solves use `chain`.
    ChainHost dhchain;
    bool use_dh = false;
    float* aux_dh = nullptr;
    const ChainHost& solve_chain() const { return use_dh ? dhchain : chain; }
    int family = IKPSO_KERNEL_RESIDENT;
    int requested = IKPSO_KERNEL_AUTO;
    std::string kname;     // kernel family / topology, for ikpso_solver_kernel_name
    std::string kname_latency;  // the cooperative latency variant AUTO may pick per call
    bool last_latency = false;  // the last solve_batch ran the latency variant
    void* ws = nullptr;    // streaming / cooperative workspace
    size_t ws_bytes = 0;
    int P = 0;
    int mode = IKPSO_ARITH_FAST;
    ikpso_rng_state* rng = nullptr;
    int64_t capacity = 0;
    // Cooperative solves: the generator states as they were before the launch,
    // and what ikpso_solver_sync needs to re-run the batch on the streaming
    // kernels if a group could not assemble.
    ikpso_rng_state* rng_snap = nullptr;
    int64_t snap_capacity = 0;
    struct {
        bool active = false;
        const float* targets = nullptr;
        const float* start_pose = nullptr;
        int64_t num_swarms = 0;
        int32_t iterations = 0;
        float *out_angles = nullptr, *out_fitness = nullptr, *out_residual = nullptr;
        hipStream_t stream = nullptr;
    } pending;
    int64_t fallbacks = 0;
    // a cooperative solve's error flag, in coherent pinned memory the kernel writes
    // (read by ikpso_solver_sync after its synchronisation), and its device address
    int32_t* err_host = nullptr;
    int32_t* err_dev = nullptr;
    CoopSlotState slots;  // the cooperative slots in `ws` between solves
#if IKPSO_COOP_TIMING
    unsigned long long* pending_timing = nullptr;
    int pending_timing_n = 0;
#endif
};

namespace {

// Grow a device buffer to at least `need` bytes (contents not kept).
ikpso_status grow(void** buf, size_t* have, size_t need)
{
    if (need <= *have) return IKPSO_OK;
    if (*buf) IKPSO_HIP(hipFree(*buf));  // hipFree synchronises the device
    *buf = nullptr;
    *have = 0;
    IKPSO_HIP(hipMalloc(buf, need));
    *have = need;
    return IKPSO_OK;
}

// The batch on the streaming kernels (state in HBM, I + 2 launches; no
// co-residency requirement).
ikpso_status solve_streaming(ikpso_solver* s, void** ws, size_t* ws_bytes, const float* targets,
                             const float* start_pose, int64_t num_swarms, int32_t iterations, float* out_angles,
                             float* out_fitness, float* out_residual, hipStream_t hs)
{
    const ChainHost& ch = s->solve_chain();
    const int D = ch.kernel_dims();
    s->slots.invalidate();  // the streaming workspace overwrites the cooperative slots
    ikpso_status st = grow(ws, ws_bytes, stream_workspace_bytes(num_swarms, s->P, D, true));
    if (st != IKPSO_OK) return st;
    StreamIO io{};
    carve_stream(io, *ws, num_swarms, s->P, D, true);
    io.rng_aos = s->rng;
    io.targets = targets;
    io.start_pose = start_pose;
    io.out_angles = out_angles;
    io.out_fitness = out_fitness;
    io.out_residual = out_residual;
    IKPSO_HIP(launch_stream(ch, s->mode, io, iterations, hs));
    return IKPSO_OK;
}

}  // namespace

extern "C" {

int ikpso_abi_version(void) { return IKPSO_ABI_VERSION; }

const char* ikpso_build_id(void) { return ikpso_build_id_string; }

int ikpso_last_hip_error(void) { return g_last_hip_error; }

const char* ikpso_status_string(ikpso_status s)
{
    switch (s) {
    case IKPSO_OK: return "ok";
    case IKPSO_ERR_INVALID_ARG: return "invalid argument";
    case IKPSO_ERR_UNSUPPORTED: return "unsupported configuration";
    case IKPSO_ERR_HIP: return "HIP runtime error";
    case IKPSO_ERR_NO_MEMORY: return "out of device memory";
    default: return "unknown status";
    }
}

ikpso_status ikpso_init_generators_seeded(ikpso_rng_state* randoms, int64_t count, uint64_t seed_base, void* stream)
{
    if (count < 0 || (count > 0 && !randoms)) return IKPSO_ERR_INVALID_ARG;
    IKPSO_HIP(launch_init_generators(randoms, count, seed_base, (hipStream_t)stream));
    return IKPSO_OK;
}

// initGenerators (src/utility_kernels.cuh:33-47): launch, then synchronise.
ikpso_status ikpso_init_generators(ikpso_rng_state* randoms, int size, void* stream)
{
    ikpso_status s = ikpso_init_generators_seeded(randoms, size, 0, stream);
    if (s != IKPSO_OK) return s;
    IKPSO_HIP(hipStreamSynchronize((hipStream_t)stream));
    return IKPSO_OK;
}

ikpso_status ikpso_calculate_pso(float* particles, const float* positions, float* bests, ikpso_rng_state* randoms,
                                 int size, const ikpso_node* chain, int node_count, ikpso_pso_config pso,
                                 ikpso_fitness_config fit, float* result, const ikpso_collider* colliders,
                                 int collider_count, void* stream)
{
    if (collider_count < 0 || (collider_count > 0 && !colliders)) return IKPSO_ERR_INVALID_ARG;
    if (size <= 0 || !particles || !bests || !randoms || !chain || !result || node_count < 2 ||
        node_count - 1 > kMaxJoints || pso.iterations < 0)
        return IKPSO_ERR_INVALID_ARG;
    IKPSO_HIP(take_pending_error());
    std::vector<ikpso_node> nodes(node_count);
    ikpso_status st = fetch_any(nodes.data(), chain, sizeof(ikpso_node) * node_count);
    if (st != IKPSO_OK) return st;
    const int J = node_count - 1, D = 3 * J;
    std::vector<float> pos;
    Extras ex;
    if (fit.distance_weight != 0.0f && positions) {
        const char* ps = getenv("IKPSO_POSREF");
        ex.posref_node_slot = ps && strcmp(ps, "node_slot") == 0;
        const size_t n = 4 * (size_t)(ex.posref_node_slot ? J + 2 : J);
        pos.resize(n);
        st = fetch_any(pos.data(), positions, sizeof(float) * n);
        if (st != IKPSO_OK) return st;
        ex.positions = pos.data();
    }
    std::vector<ikpso_collider> boxes(collider_count);
    if (collider_count > 0) {
        st = fetch_any(boxes.data(), colliders, sizeof(ikpso_collider) * collider_count);
        if (st != IKPSO_OK) return st;
        ex.colliders = boxes.data();
        ex.collider_count = collider_count;
    }
    ChainHost ch;
    st = parse_chain(nodes, pso, fit, ex, ch);
    if (st != IKPSO_OK) return st;
    // The reference-compatible entry has no mode argument; IKPSO_ARITH=reference
    // selects the reference's operation order (parity runs).
    const char* env = getenv("IKPSO_ARITH");
    const int mode = (env && strcmp(env, "reference") == 0) ? IKPSO_ARITH_REFERENCE : IKPSO_ARITH_FAST;
    const int family = pick_kernel(ch, mode, size, env_kernel());
    if (family < 0) return IKPSO_ERR_UNSUPPORTED;
    int family_run = family;
    if (family == IKPSO_KERNEL_RESIDENT && env_kernel() == IKPSO_KERNEL_AUTO && prefer_latency_coop(ch, mode, size, 1))
        family_run = IKPSO_KERNEL_COOP;
    int cg = 0, cng = 0, cblk = 0;
    bool clin = false;
    if (family_run == IKPSO_KERNEL_COOP &&
        !coop_plan(ch, mode, size, 1, env_kernel() == IKPSO_KERNEL_AUTO, &cg, &cng, &cblk, &clin))
        return IKPSO_ERR_UNSUPPORTED;

    std::lock_guard<std::mutex> lk(g_scratch_mu);
    // device scratch: [aux (at float ceil64(D)) | workspace]; aux is uploaded here (when
    // it changed) and the call synchronises before returning, so `ch.aux` outlives
    // every use.  The cooperative path also keeps a snapshot of the generator
    // states (written by the kernel as it loads them) and room for the streaming
    // fallback.  The answer goes to `result` directly when that is device memory,
    // else to the pinned block, copied out after the synchronisation.
    const size_t aux_at = ((size_t)D + 63) & ~size_t(63);
    const size_t head = sizeof(float) * (aux_at + ch.aux.size());
    const size_t sws = stream_workspace_bytes(1, size, D, false);
    const size_t snap = ((sizeof(ikpso_rng_state) * (size_t)size + 255) & ~size_t(255));
    const size_t cws = family_run == IKPSO_KERNEL_COOP ? ((coop_workspace_bytes(cng, cg, D, cblk) + 255) & ~size_t(255)) : 0;
    const size_t ws = family_run == IKPSO_KERNEL_STREAMING ? sws
                      : family_run == IKPSO_KERNEL_COOP ? cws + snap + sws
                                                          : 0;
    float* dres = nullptr;
    st = scratch(((head + 255) & ~size_t(255)) + ws, &dres);
    if (st != IKPSO_OK) return st;
    if (!g_frame.pinned) {
        void* h = nullptr;
        IKPSO_HIP(hipHostMalloc(&h, sizeof(int32_t) * kFramePinnedWords, hipHostMallocCoherent | hipHostMallocMapped));
        void* dv = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&dv, h, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(h);
            IKPSO_HIP(e);
        }
        g_frame.pinned = static_cast<int32_t*>(h);
        g_frame.pinned_dev = static_cast<int32_t*>(dv);
    }
    const bool direct = is_device_memory(result);
    float* const out = direct ? result : reinterpret_cast<float*>(g_frame.pinned_dev + 64);
    const hipStream_t s = (hipStream_t)stream;
    // the cached block is compared byte for byte (a value comparison would take -0 for +0 and
    // never match a NaN)
    if (g_frame.aux_at != dres + aux_at || g_frame.aux.size() != ch.aux.size() ||
        (!ch.aux.empty() && memcmp(g_frame.aux.data(), ch.aux.data(), sizeof(float) * ch.aux.size()) != 0)) {
        IKPSO_HIP(hipMemcpyAsync(dres + aux_at, ch.aux.data(), sizeof(float) * ch.aux.size(), hipMemcpyHostToDevice, s));
        g_frame.aux_at = dres + aux_at;
        g_frame.aux = ch.aux;
    }
    ch.aux_dev = dres + aux_at;
    char* const wsb = reinterpret_cast<char*>(dres) + ((head + 255) & ~size_t(255));
    if (family_run != IKPSO_KERNEL_COOP) g_frame.slots.invalidate();  // the streaming workspace overwrites the slots
    if (family_run == IKPSO_KERNEL_RESIDENT) {
        SwarmIO io{};
        io.rng = randoms;
        io.out_angles = out;
        io.dump_particles = particles;
        io.dump_bests = bests;
        io.P = size;
        io.iterations = pso.iterations;
        io.num_swarms = 1;
        IKPSO_HIP(launch_resident(ch, mode, io, s));
    } else if (family_run == IKPSO_KERNEL_COOP) {
        SwarmIO io{};
        io.rng = randoms;
        io.out_angles = out;
        io.dump_particles = particles;
        io.dump_bests = bests;
        io.P = size;
        io.iterations = pso.iterations;
        io.num_swarms = 1;
        ikpso_rng_state* const rsnap = reinterpret_cast<ikpso_rng_state*>(wsb + cws);
        io.rng_snap = rsnap;  // one swarm, started by its group: the snapshot is complete
        size_t zero = 0;
        IKPSO_HIP(carve_coop(io, wsb, cg, cng, cblk, D, s, clin, false, &zero));
        IKPSO_HIP(g_frame.slots.begin(io, wsb, zero, (uint64_t)pso.iterations + 1, s));  // one swarm: I + 1 exchanges
        io.coop_error = g_frame.pinned_dev;
        __atomic_store_n(g_frame.pinned, 0, __ATOMIC_RELEASE);
        IKPSO_HIP(launch_coop(ch, mode, io, s));
        IKPSO_HIP(hipStreamSynchronize(s));
        if (__atomic_load_n(g_frame.pinned, __ATOMIC_ACQUIRE) != 0) {
            // The group could not assemble (other work held CUs): restore the
            // generator states and solve on the streaming kernels, which need
            // no co-residency -- the caller never sees the contention.
            IKPSO_HIP(hipMemcpyAsync(randoms, rsnap, sizeof(ikpso_rng_state) * (size_t)size, hipMemcpyDeviceToDevice,
                                     s));
            StreamIO sio{};
            carve_stream(sio, reinterpret_cast<char*>(rsnap) + snap, 1, size, D, false);
            sio.state = particles;
            sio.pbf = bests;
            sio.rng_aos = randoms;
            sio.out_angles = out;
            IKPSO_HIP(launch_stream(ch, mode, sio, pso.iterations, s));
            g_coop_fallbacks.fetch_add(1);
            IKPSO_HIP(hipStreamSynchronize(s));
        }
    } else {
        StreamIO io{};
        carve_stream(io, wsb, 1, size, D, false);
        io.state = particles;  // the reference's own [3][D][P] layout is the streaming state
        io.pbf = bests;
        io.rng_aos = randoms;
        io.out_angles = out;
        IKPSO_HIP(launch_stream(ch, mode, io, pso.iterations, s));
    }
    if (family_run != IKPSO_KERNEL_COOP) IKPSO_HIP(hipStreamSynchronize(s));
    if (!direct) memcpy(result, g_frame.pinned + 64, sizeof(float) * D);
    return IKPSO_OK;
}

ikpso_status ikpso_solver_create(const ikpso_solver_desc* desc, ikpso_solver** out)
{
    if (!desc || !out || !desc->chain || desc->node_count < 2 || desc->node_count - 1 > kMaxJoints ||
        desc->particles <= 0)
        return IKPSO_ERR_INVALID_ARG;
    if (desc->arith != IKPSO_ARITH_FAST && desc->arith != IKPSO_ARITH_REFERENCE) return IKPSO_ERR_INVALID_ARG;
    *out = nullptr;
    // a caller's pending error is reported here, before fetch_any's own lookups
    // (which clear the errors they cause) could discard it
    IKPSO_HIP(take_pending_error());
    const int J = desc->node_count - 1;
    std::vector<ikpso_node> nodes(desc->node_count);
    ikpso_status st = fetch_any(nodes.data(), desc->chain, sizeof(ikpso_node) * desc->node_count);
    if (st != IKPSO_OK) return st;
    std::vector<float> pos, slo, shi;
    std::vector<uint8_t> mask;
    Extras ex;
    int D = 3 * J;  // free dimensions
    if (desc->axis_mask) {
        mask.resize(desc->node_count);
        if ((st = fetch_any(mask.data(), desc->axis_mask, mask.size())) != IKPSO_OK) return st;
        ex.axis_mask = mask.data();
        D = 0;
        for (int k = 1; k <= J; ++k) D += __builtin_popcount(mask[k] & 7u);
    }
    if (desc->fit.distance_weight != 0.0f && desc->positions) {
        ex.posref_node_slot = (desc->flags & IKPSO_FLAG_POSREF_NODE_SLOT) != 0;
        const size_t n = 4 * (size_t)(ex.posref_node_slot ? J + 2 : J);
        pos.resize(n);
        if ((st = fetch_any(pos.data(), desc->positions, sizeof(float) * n)) != IKPSO_OK) return st;
        ex.positions = pos.data();
    }
    if (desc->limit_weight != 0.0f) {
        if (!desc->soft_lo || !desc->soft_hi) return IKPSO_ERR_INVALID_ARG;
        slo.resize(D);
        shi.resize(D);
        if ((st = fetch_any(slo.data(), desc->soft_lo, sizeof(float) * D)) != IKPSO_OK) return st;
        if ((st = fetch_any(shi.data(), desc->soft_hi, sizeof(float) * D)) != IKPSO_OK) return st;
        ex.limit_weight = desc->limit_weight;
        ex.soft_lo = slo.data();
        ex.soft_hi = shi.data();
    }
    std::vector<ikpso_collider> boxes;
    if (desc->collider_count < 0 || (desc->collider_count > 0 && !desc->colliders)) return IKPSO_ERR_INVALID_ARG;
    if (desc->collider_count > 0) {
        boxes.resize(desc->collider_count);
        if ((st = fetch_any(boxes.data(), desc->colliders, sizeof(ikpso_collider) * boxes.size())) != IKPSO_OK)
            return st;
        ex.colliders = boxes.data();
        ex.collider_count = desc->collider_count;
    }
    ikpso_solver* s = new (std::nothrow) ikpso_solver();
    if (!s) return IKPSO_ERR_NO_MEMORY;
    st = parse_chain(nodes, desc->pso, desc->fit, ex, s->chain);
    if (st != IKPSO_OK) {
        delete s;
        return st;
    }
    s->P = desc->particles;
    s->mode = desc->arith;
    // FAST solves of a masked serial chain run on its folded form
    s->use_dh = s->mode == IKPSO_ARITH_FAST && !(desc->flags & IKPSO_FLAG_NO_FOLD) &&
                build_dh(nodes, s->chain, ex, s->dhchain);
    {
        const size_t bytes = sizeof(float) * s->chain.aux.size();
        hipError_t e = hipMalloc(&s->aux, bytes);
        if (e == hipSuccess) e = hipMemcpy(s->aux, s->chain.aux.data(), bytes, hipMemcpyHostToDevice);
        if (e == hipSuccess && s->use_dh) {
            const size_t b2 = sizeof(float) * s->dhchain.aux.size();
            e = hipMalloc(&s->aux_dh, b2);
            if (e == hipSuccess) e = hipMemcpy(s->aux_dh, s->dhchain.aux.data(), b2, hipMemcpyHostToDevice);
        }
        if (e != hipSuccess) {
            if (s->aux) (void)hipFree(s->aux);
            if (s->aux_dh) (void)hipFree(s->aux_dh);
            delete s;
            return hip_status(e);
        }
        s->chain.aux_dev = s->aux;
        s->dhchain.aux_dev = s->aux_dh;
    }
    const ChainHost& sch = s->solve_chain();
    s->family = pick_kernel(sch, s->mode, s->P, desc->kernel);
    s->requested = desc->kernel;
    if (s->family >= 0) s->kname = kernel_name(sch, s->family);
    if (s->family >= 0)
        s->kname_latency = kernel_name(sch, IKPSO_KERNEL_COOP) +
                           (coop_latency_split(sch) ? " (latency variant, generator waves)" : " (latency variant)");
    if (s->family < 0 || desc->kernel < IKPSO_KERNEL_AUTO || desc->kernel > IKPSO_KERNEL_COOP) {
        (void)hipFree(s->aux);
        if (s->aux_dh) (void)hipFree(s->aux_dh);
        delete s;
        return (desc->kernel == IKPSO_KERNEL_RESIDENT || desc->kernel == IKPSO_KERNEL_COOP) ? IKPSO_ERR_UNSUPPORTED
                                                                                              : IKPSO_ERR_INVALID_ARG;
    }
    *out = s;
    return IKPSO_OK;
}

ikpso_status ikpso_solver_destroy(ikpso_solver* s)
{
    if (!s) return IKPSO_OK;
    // a pending cooperative solve still runs on the buffers freed below: settle it
    // (its fallback, if it needs one, completes the caller's outputs)
    const ikpso_status pend = s->pending.active ? ikpso_solver_sync(s) : IKPSO_OK;
    if (s->rng) (void)hipFree(s->rng);
    if (s->rng_snap) (void)hipFree(s->rng_snap);
    if (s->err_host) (void)hipHostFree(s->err_host);
    if (s->aux) (void)hipFree(s->aux);
    if (s->aux_dh) (void)hipFree(s->aux_dh);
    if (s->ws) (void)hipFree(s->ws);
    delete s;
    return pend;
}

ikpso_status ikpso_solver_seed(ikpso_solver* s, int64_t capacity, uint64_t seed_base, int64_t first_swarm,
                               void* stream)
{
    if (!s || capacity < 0 || first_swarm < 0) return IKPSO_ERR_INVALID_ARG;
    if (s->pending.active) {  // settle the last cooperative solve before its states are replaced
        const ikpso_status st = ikpso_solver_sync(s);
        if (st != IKPSO_OK) return st;
    }
    if (capacity > s->capacity) {
        if (s->rng) IKPSO_HIP(hipFree(s->rng));
        s->rng = nullptr;
        s->capacity = 0;
        IKPSO_HIP(hipMalloc(&s->rng, sizeof(ikpso_rng_state) * (size_t)capacity * s->P));
        s->capacity = capacity;
    }
    IKPSO_HIP(launch_init_generators(s->rng, capacity * s->P, seed_base + (uint64_t)first_swarm * s->P,
                                     (hipStream_t)stream));
    return IKPSO_OK;
}

ikpso_status ikpso_solve_batch(ikpso_solver* s, const float* targets, const float* start_pose, int64_t num_swarms,
                               int32_t iterations, float* out_angles, float* out_fitness, float* out_residual,
                               void* stream)
{
    if (!s || num_swarms < 0 || iterations < 0) return IKPSO_ERR_INVALID_ARG;
    if (num_swarms == 0) return IKPSO_OK;
    if (!out_angles) return IKPSO_ERR_INVALID_ARG;  // targets == NULL: chain targets for every swarm
    if (num_swarms > s->capacity || !s->rng) return IKPSO_ERR_INVALID_ARG;  // seed first
    if (num_swarms > 0x7fffffff) return IKPSO_ERR_INVALID_ARG;
    IKPSO_HIP(take_pending_error());
    const hipStream_t hs = (hipStream_t)stream;
    if (s->pending.active) {  // the previous cooperative solve was not synced: settle it first
        const ikpso_status st = ikpso_solver_sync(s);
        if (st != IKPSO_OK) return st;
    }
    const ChainHost& ch = s->solve_chain();
    const bool latency_coop = s->family == IKPSO_KERNEL_RESIDENT && s->requested == IKPSO_KERNEL_AUTO &&
                              prefer_latency_coop(ch, s->mode, s->P, num_swarms);
    s->last_latency = latency_coop;
    if (s->family == IKPSO_KERNEL_RESIDENT && !latency_coop) {
        SwarmIO io{};
        io.targets = targets;
        io.start_pose = start_pose;
        io.rng = s->rng;
        io.out_angles = out_angles;
        io.out_fitness = out_fitness;
        io.out_residual = out_residual;
        io.P = s->P;
        io.iterations = iterations;
        io.num_swarms = num_swarms;
        IKPSO_HIP(launch_resident(ch, s->mode, io, hs));
        return IKPSO_OK;
    }
    const int D = ch.kernel_dims();
    if (s->family == IKPSO_KERNEL_COOP || latency_coop) {
        int G, NG, T;
        bool linear = false;
        if (!coop_plan(ch, s->mode, s->P, num_swarms, s->requested == IKPSO_KERNEL_AUTO, &G, &NG, &T, &linear))
            return IKPSO_ERR_UNSUPPORTED;
        const size_t had = s->ws_bytes;
        ikpso_status st = grow(&s->ws, &s->ws_bytes, coop_workspace_bytes(NG, G, D, T));
        if (st != IKPSO_OK) return st;
        if (s->ws_bytes != had) s->slots.invalidate();  // a new allocation: contents unknown
        if (!s->err_host) {
            void* h = nullptr;
            IKPSO_HIP(hipHostMalloc(&h, sizeof(int32_t), hipHostMallocCoherent | hipHostMallocMapped));
            void* dv = nullptr;
            const hipError_t e = hipHostGetDevicePointer(&dv, h, 0);
            if (e != hipSuccess) {
                (void)hipHostFree(h);
                IKPSO_HIP(e);
            }
            s->err_host = static_cast<int32_t*>(h);
            s->err_dev = static_cast<int32_t*>(dv);
        }
        // snapshot of the generator states the launch starts from (48 B per
        // particle): the fallback re-runs the batch from it.  One swarm: the kernel
        // writes it as its chunks load the states; more: one D2D copy before the
        // launch (a group that gives up never loads its later swarms)
        if (num_swarms > s->snap_capacity) {
            if (s->rng_snap) IKPSO_HIP(hipFree(s->rng_snap));
            s->rng_snap = nullptr;
            s->snap_capacity = 0;
            IKPSO_HIP(hipMalloc(&s->rng_snap, sizeof(ikpso_rng_state) * (size_t)s->capacity * s->P));
            s->snap_capacity = s->capacity;
        }
        if (num_swarms > 1)
            IKPSO_HIP(hipMemcpyAsync(s->rng_snap, s->rng, sizeof(ikpso_rng_state) * (size_t)num_swarms * s->P,
                                     hipMemcpyDeviceToDevice, hs));
        SwarmIO io{};
        io.rng_snap = num_swarms == 1 ? s->rng_snap : nullptr;
        io.targets = targets;
        io.start_pose = start_pose;
        io.rng = s->rng;
        io.out_angles = out_angles;
        io.out_fitness = out_fitness;
        io.out_residual = out_residual;
        io.P = s->P;
        io.iterations = iterations;
        io.num_swarms = num_swarms;
        size_t zero = 0;
        IKPSO_HIP(carve_coop(io, s->ws, G, NG, T, D, hs, linear, false, &zero));
        // a group runs at most every swarm: B (I + 1) exchanges bound its numbering
        IKPSO_HIP(s->slots.begin(io, static_cast<char*>(s->ws), zero, (uint64_t)num_swarms * ((uint64_t)iterations + 1), hs));
        io.coop_error = s->err_dev;
        *s->err_host = 0;  // the previous solve has settled: nothing writes it now
        // the reported name follows the variant that runs (long chains' throughput chunks are
        // kCoopLatencyThreads wide too: only a block other than the throughput one is the latency plan)
        CoopGeometry geo;
        s->last_latency = coop_geometry(ch, s->mode, &geo) && T != geo.threads;
        IKPSO_HIP(launch_coop(ch, s->mode, io, hs));
        s->pending.active = true;
        s->pending.targets = targets;
        s->pending.start_pose = start_pose;
        s->pending.num_swarms = num_swarms;
        s->pending.iterations = iterations;
        s->pending.out_angles = out_angles;
        s->pending.out_fitness = out_fitness;
        s->pending.out_residual = out_residual;
        s->pending.stream = hs;
#if IKPSO_COOP_TIMING
        s->pending_timing = io.coop_timing;
        s->pending_timing_n = NG * G;
#endif
        return IKPSO_OK;
    }
    return solve_streaming(s, &s->ws, &s->ws_bytes, targets, start_pose, num_swarms, iterations, out_angles,
                           out_fitness, out_residual, hs);
}

ikpso_status ikpso_solver_sync(ikpso_solver* s)
{
    if (!s) return IKPSO_ERR_INVALID_ARG;
    if (!s->pending.active) return IKPSO_OK;
    auto& p = s->pending;
    // `pending` stays active until the flag has been read and, if a group gave
    // up, the fallback has run: a failure on the way (an allocation, a copy)
    // returns its error and leaves the solve pending, so the next sync, solve or
    // generator_states call settles it instead of reporting OK over NaN answers.
    // the kernel writes the flag into coherent pinned memory: one synchronisation
    IKPSO_HIP(hipStreamSynchronize(p.stream));
    const int32_t err = __atomic_load_n(s->err_host, __ATOMIC_ACQUIRE);
#if IKPSO_COOP_TIMING
    if (s->pending_timing) {  // measurement build: mean cycles per iteration over the workgroups
        std::vector<unsigned long long> t((size_t)s->pending_timing_n * 8);
        IKPSO_HIP(hipMemcpy(t.data(), s->pending_timing, t.size() * 8, hipMemcpyDeviceToHost));
        double a = 0, b = 0, c = 0, it = 0, imp = 0, rem = 0, pol = 0, ah = 0;
        for (size_t i = 0; i < t.size(); i += 8)
            a += t[i], b += t[i + 1], it += t[i + 2], c += t[i + 3], imp += t[i + 4], rem += t[i + 5],
                pol += t[i + 6], ah += t[i + 7];
        fprintf(stderr,
                "ikpso coop timing: %d workgroups, per iteration (wave 0): step %.0f, argmin barrier %.0f, "
                "hand-off %.0f cycles (of which publish + draws ahead %.0f); improving exchanges %.3f (won by "
                "another chunk %.3f), key polls %.2f\n",
                s->pending_timing_n, a / it, c / it, b / it, ah / it, imp / it, rem / it, pol / it);
    }
#endif
    if (!err) {
        p.active = false;
        return IKPSO_OK;
    }
    // A group gave up waiting for its members (the GPU is shared): restore the
    // generator states and solve the whole batch on the streaming kernels.
    IKPSO_HIP(hipMemcpyAsync(s->rng, s->rng_snap, sizeof(ikpso_rng_state) * (size_t)p.num_swarms * s->P,
                             hipMemcpyDeviceToDevice, p.stream));
    // the cooperative workspace is idle now (the launch has completed): the
    // streaming solve runs in it, grown as needed, so no second workspace is held
    const ikpso_status st = solve_streaming(s, &s->ws, &s->ws_bytes, p.targets, p.start_pose, p.num_swarms,
                                            p.iterations, p.out_angles, p.out_fitness, p.out_residual, p.stream);
    if (st != IKPSO_OK) return st;
    IKPSO_HIP(hipStreamSynchronize(p.stream));
    p.active = false;
    ++s->fallbacks;
    g_coop_fallbacks.fetch_add(1);
    return IKPSO_OK;
}

int64_t ikpso_solver_fallbacks(const ikpso_solver* s) { return s ? s->fallbacks : 0; }

ikpso_status ikpso_solver_generator_states(ikpso_solver* s, int64_t first_swarm, int64_t count, void* dst, void* stream)
{
    if (!s || first_swarm < 0 || count < 0 || (count > 0 && !dst) || first_swarm + count > s->capacity)
        return IKPSO_ERR_INVALID_ARG;
    if (s->pending.active) {
        const ikpso_status st = ikpso_solver_sync(s);
        if (st != IKPSO_OK) return st;
    }
    if (count == 0) return IKPSO_OK;
    const hipStream_t hs = (hipStream_t)stream;
    IKPSO_HIP(hipMemcpyAsync(dst, s->rng + (size_t)first_swarm * s->P, sizeof(ikpso_rng_state) * (size_t)count * s->P,
                             hipMemcpyDefault, hs));
    IKPSO_HIP(hipStreamSynchronize(hs));
    return IKPSO_OK;
}

int64_t ikpso_coop_fallbacks(void) { return g_coop_fallbacks.load(); }

ikpso_status ikpso_solver_evaluate(ikpso_solver* s, const float* angles, const float* targets, const float* rest,
                                   int64_t n, float* out_fitness, float* out_positions, void* stream)
{
    if (!s || n < 0 || (n > 0 && !angles)) return IKPSO_ERR_INVALID_ARG;
    EvalIO io{angles, targets, rest, out_fitness, out_positions, n};
    IKPSO_HIP(launch_evaluate(s->chain, s->mode, io, (hipStream_t)stream));
    return IKPSO_OK;
}

int ikpso_solver_dof(const ikpso_solver* s) { return s ? s->chain.dof() : 0; }
int ikpso_solver_effectors(const ikpso_solver* s) { return s ? s->chain.E : 0; }
int ikpso_solver_collider_count(const ikpso_solver* s) { return s ? s->chain.num_coll : 0; }
const char* ikpso_solver_kernel_name(const ikpso_solver* s)
{
    return s ? (s->last_latency ? s->kname_latency : s->kname).c_str() : "";
}

}  // extern "C"
