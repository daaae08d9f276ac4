// ikpso_collide.h -- the collider term of the fitness on gfx950: box-box GJK
// intersection of every node box and link box of a particle's arm against the
// scene's colliders (calculateDistance, src/kernel.cu:104-136; any hit makes
// the fitness FLT_MAX).
//
// Reference arithmetic restated (src/ = InverseKinematicsResearch/InverseKinematicsResearch/):
//   matrixToQuaternion          src/matrix_operations.cuh:78-109
//   supportBox / SupportCalc    src/kernel.cu:499-530,594-612 (firstDir = (1,1,0))
//   GJK                         src/kernel.cu:538-592 (GJK_ITERATIONS = 50, src/ik_constants.h)
//   doSimplex2/3/4              src/kernel.cu:631-870
//   Vec3PointTriDist2 / PointSegmentDist src/kernel.cu:872-1010
//   quatRotVec / quatInvert     src/kernel.cu:1012-1061
// Every operation keeps the reference's order and rounding (no FMA
// contraction, matrixToQuaternion's sqrt in fp64) in both arithmetic modes, so
// for the same frames the hit/no-hit decision is the reference's bit for bit.
//
// MI355X shape: one lane = one particle, so the test is per lane and the
// simplex lives in registers (four named points, permuted explicitly instead
// of the reference's indexed array, which would go to scratch).  Colliders are
// uniform across the workgroup: their records (with the inverse quaternion
// and bounding radius precomputed on the host) are read through scalar loads.
// A bounding-sphere test skips GJK for box pairs whose support points cannot
// come within 1e-3 of each other -- GJK can only report an intersection when
// the origin is within sqrt(FLT_EPSILON) (3.5e-4) of a simplex of Minkowski
// support points, all of which lie inside the two spheres' Minkowski ball --
// so the early-out never changes the answer, and the (wave-divergent, up to
// 50-iteration) GJK loop runs only for lanes whose arm is near a collider.
// The sphere test runs twice: first inline in the fitness's FK pass, on the
// node's position and a radius bound that needs no quaternion (near_collider),
// which keeps the frames of the nodes that pass it; then, after the pass and only
// for those nodes, out of line with the node's quaternion (node_collides, one call
// site: FitnessAcc::finish).  node_collides is a leaf function -- GJK and its
// distance tests inlined at one site -- so a call saves no registers of its own
// around nested calls.
#pragma once

#include <hip/hip_runtime.h>

#include <float.h>

namespace ikpso {

// Device collider record (built by the host from obj_t, src/BoxCollider.h:4-10).
struct CollRec {
    float px, py, pz;      // centre
    float qx, qy, qz, qw;  // orientation quaternion (as given)
    float ix, iy, iz, iw;  // quatInvert2 of it (copy when |q|^2 < FLT_EPSILON)
    float sx, sy, sz;      // full edge lengths (obj_t x, y, z)
    float radius;          // bound on |support point - centre| (see sphere_radius)
    float pad_;
};
static_assert(sizeof(CollRec) == 64, "collider record is 16 floats");

constexpr int kGjkIterations = 50;      // GJK_ITERATIONS

// IKPSO_COLLIDE_STATS builds (tools/collide_stats.py; variants/, never shipped)
// count, per solve, what the collider term does -- lane counts unless noted:
enum {
    kCsPre = 0,      // node/collider pairs through the inline sphere test (near_collider)
    kCsPrePass,      // ... that pass it
    kCsExact,        // pairs through the quaternion sphere test (node_collides)
    kCsExactPass,    // ... that pass it (GJK calls)
    kCsGjkIter,      // GJK loop trips, summed over lanes
    kCsGjkWaveIter,  // GJK loop trips, summed over waves (what the SIMD executes)
    kCsGjkHit,       // GJK calls that report an intersection
    kCsCalls,        // node_collides calls, summed over waves
    kCsCount
};
#ifndef IKPSO_COLLIDE_STATS
#define IKPSO_COLLIDE_STATS 0
#endif
#if IKPSO_COLLIDE_STATS
#define IKPSO_CS_PARAM , unsigned long long* cs
#define IKPSO_CS_ARG , cs
// add the number of active lanes with `pred` to counter i (one atomic per wave)
__device__ __forceinline__ void cs_count(unsigned long long* cs, int i, bool pred)
{
    const unsigned long long active = __builtin_amdgcn_read_exec();
    const unsigned long long m = __builtin_amdgcn_ballot_w64(pred);
    if (cs && (int)__lane_id() == __builtin_ctzll(active)) atomicAdd(&cs[i], (unsigned long long)__builtin_popcountll(m));
}
#else
#define IKPSO_CS_PARAM
#define IKPSO_CS_ARG
#endif
constexpr float kGizmo = 0.2f;          // GIZMO_SIZE

struct V3 {
    float x, y, z;
};

#pragma clang fp contract(off)

__host__ __device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__host__ __device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__host__ __device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__host__ __device__ __forceinline__ V3 neg(V3 a) { return v3(a.x * -1.0f, a.y * -1.0f, a.z * -1.0f); }
__host__ __device__ __forceinline__ V3 scale(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
// float3Dot: ((x*x') + y*y') + z*z'
__host__ __device__ __forceinline__ float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__host__ __device__ __forceinline__ V3 cross(V3 a, V3 b)
{
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__host__ __device__ __forceinline__ bool is_zero(float v) { return (v > 0.0f ? v : -v) < FLT_EPSILON; }
__host__ __device__ __forceinline__ int signum(float v) { return is_zero(v) ? 0 : (v < 0.0f ? -1 : 1); }
__host__ __device__ __forceinline__ bool nonneg(float v) { return is_zero(v) || v > 0.0f; }  // IsZERO || > 0
__host__ __device__ __forceinline__ bool veq(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

// quatRotVec (src/kernel.cu:1012-1037), expanded form and order.
__host__ __device__ __forceinline__ V3 quat_rot(V3 v, float x, float y, float z, float w)
{
    const float c1x = y * v.z - z * v.y + w * v.x;
    const float c1y = z * v.x - x * v.z + w * v.y;
    const float c1z = x * v.y - y * v.x + w * v.z;
    const float c2x = y * c1z - z * c1y;
    const float c2y = z * c1x - x * c1z;
    const float c2z = x * c1y - y * c1x;
    return v3(v.x + 2.0f * c2x, v.y + 2.0f * c2y, v.z + 2.0f * c2z);
}

// quatInvert2 (src/kernel.cu:1039-1061).
__host__ __device__ __forceinline__ void quat_inverse(const float q[4], float out[4])
{
    out[0] = q[0];
    out[1] = q[1];
    out[2] = q[2];
    out[3] = q[3];
    float l2 = ((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3];
    if (l2 < FLT_EPSILON) return;
    l2 = 1.0f / l2;
    out[0] = -q[0] * l2;
    out[1] = -q[1] * l2;
    out[2] = -q[2] * l2;
    out[3] = q[3] * l2;
}

// Largest |quatRotVec(v, q)| / |v|: quatRotVec is the linear map
// (1 - 2|r|^2) I + 2 r r^T + 2w [r]x (r = q.xyz), with singular values 1 and
// sqrt((1 - 2|r|^2)^2 + 4 w^2 |r|^2) (1 for a unit quaternion).
__host__ __device__ __forceinline__ float quat_gain(float x, float y, float z, float w)
{
    const float r2 = x * x + y * y + z * z;
    const float a = 1.0f - 2.0f * r2;
    const float g = sqrtf(a * a + 4.0f * w * w * r2);
    return (g > 1.0f ? g : 1.0f) * (1.0f + 1e-5f);
}

// Bound on |support point - centre| of a box: gain * half diagonal.
__host__ __device__ __forceinline__ float sphere_radius(float sx, float sy, float sz, float gain)
{
    return 0.5f * sqrtf(sx * sx + sy * sy + sz * sz) * gain;
}

// A box with its orientation and inverse in registers.
struct Box {
    float px, py, pz, qx, qy, qz, qw, ix, iy, iz, iw, sx, sy, sz, radius;
};

__device__ __forceinline__ Box box_from_record(const CollRec& c)
{
    return Box{c.px, c.py, c.pz, c.qx, c.qy, c.qz, c.qw, c.ix, c.iy, c.iz, c.iw, c.sx, c.sy, c.sz, c.radius};
}

// supportBox (src/kernel.cu:505-530)
__device__ __forceinline__ V3 support_box(const Box& b, V3 dir)
{
    const V3 d = quat_rot(dir, b.ix, b.iy, b.iz, b.iw);
    V3 v = v3((float)signum(d.x) * b.sx * 0.5f, (float)signum(d.y) * b.sy * 0.5f, (float)signum(d.z) * b.sz * 0.5f);
    v = quat_rot(v, b.qx, b.qy, b.qz, b.qw);
    return v + v3(b.px, b.py, b.pz);
}

// SupportCalc (src/kernel.cu:594-612)
__device__ __forceinline__ V3 support(const Box& a, const Box& b, V3 dir)
{
    return support_box(a, dir) - support_box(b, neg(dir));
}

// PointSegmentDist (src/kernel.cu:955-1010), squared; `witness` selects the
// reference's witness branch (its arithmetic differs from the plain one).
__device__ __forceinline__ float point_seg_dist2(V3 P, V3 x0, V3 b, bool witness)
{
    const V3 d = b - x0;
    const V3 a = x0 - P;
    float t = -1.0f * dot(a, d);
    t = t / dot(d, d);
    if (t < 0.0f || is_zero(t)) {
        const V3 e = x0 - P;
        return dot(e, e);
    }
    if (t > 1.0f || t == 1.0f) {
        const V3 e = b - P;
        return dot(e, e);
    }
    if (witness) {
        const V3 e = (scale(d, t) + x0) - P;
        return dot(e, e);
    }
    const V3 e = scale(d, t) + a;
    return dot(e, e);
}

// Vec3PointTriDist2 (src/kernel.cu:872-953) with witness == NULL.
__device__ __forceinline__ float point_tri_dist2(V3 P, V3 x0, V3 B, V3 C)
{
    const V3 d1 = B - x0, d2 = C - x0, a = x0 - P;
    const float u = dot(a, a), v = dot(d1, d1), w = dot(d2, d2);
    const float p = dot(a, d1), q = dot(a, d2), r = dot(d1, d2);
    const float den = w * v - r * r;
    float s = -1.0f, t = -1.0f;
    if (!is_zero(den)) {
        s = (q * r - w * p) / den;
        t = (-s * r - q) / w;
    }
    if (nonneg(s) && (s == 1.0f || s < 1.0f) && nonneg(t) && (t == 1.0f || t < 1.0f) &&
        (t + s == 1.0f || t + s < 1.0f)) {
        float dist = s * s * v;
        dist += t * t * w;
        dist += 2.0f * s * t * r;
        dist += 2.0f * s * p;
        dist += 2.0f * t * q;
        dist += u;
        return dist;
    }
    float dist = point_seg_dist2(P, x0, B, false);
    float alt = point_seg_dist2(P, x0, C, true);
    if (alt < dist) dist = alt;
    alt = point_seg_dist2(P, B, C, true);
    if (alt < dist) dist = alt;
    return dist;
}

// The simplex: s0..s(n-1), newest last (simplex_t).  doSimplex3 on the
// triangle (s0, s1, s2), A = s2; returns 1 / -1 / 0 like the reference and
// rewrites the simplex and direction.
__device__ __forceinline__ int simplex3(V3& s0, V3& s1, V3& s2, int& n, V3& dir)
{
    const V3 A = s2, B = s1, C = s0;
    if (is_zero(point_tri_dist2(v3(0.0f, 0.0f, 0.0f), A, B, C))) return 1;
    if (veq(A, B) || veq(A, C)) return -1;
    const V3 AO = neg(A);
    const V3 AB = B - A, AC = C - A;
    const V3 ABC = cross(AB, AC);
    if (nonneg(dot(cross(ABC, AC), AO))) {
        if (nonneg(dot(AC, AO))) {
            s1 = A;  // (C, A)
            n = 2;
            dir = cross(cross(AC, AO), AC);
        } else if (nonneg(dot(AB, AO))) {
            s0 = B;  // (B, A)
            s1 = A;
            n = 2;
            dir = cross(cross(AB, AO), AB);
        } else {
            s0 = A;
            n = 1;
            dir = AO;
        }
    } else if (nonneg(dot(cross(AB, ABC), AO))) {
        if (nonneg(dot(AB, AO))) {
            s0 = B;
            s1 = A;
            n = 2;
            dir = cross(cross(AB, AO), AB);
        } else {
            s0 = A;
            n = 1;
            dir = AO;
        }
    } else if (nonneg(dot(ABC, AO))) {
        dir = ABC;
    } else {
        s0 = B;  // swap B and C
        s1 = C;
        dir = neg(ABC);
    }
    return 0;
}

// GJKIntersect (src/kernel.cu:532-592): true if the boxes intersect.
__device__ __forceinline__ bool gjk_intersect(Box a, Box b IKPSO_CS_PARAM)
{
    V3 dir = v3(1.0f, 1.0f, 0.0f);  // firstDir
    V3 last = support(a, b, dir);
    V3 s0 = last, s1 = last, s2 = last, s3 = last;
    int n = 1;
    dir = neg(last);
    for (int it = 0; it < kGjkIterations; ++it) {
#if IKPSO_COLLIDE_STATS
        cs_count(cs, kCsGjkIter, true);
        cs_count(cs, kCsGjkWaveIter, (int)__lane_id() == __builtin_ctzll(__builtin_amdgcn_read_exec()));
#endif
        last = support(a, b, dir);
        if (dot(last, dir) < 0.0f) return false;
        int r;
        if (n == 1) {  // doSimplex2: A = last, B = s0
            s1 = last;
            n = 2;
            const V3 A = s1, B = s0;
            const V3 AB = B - A, AO = neg(A);
            const float d = dot(AB, AO);
            const V3 t = cross(AB, AO);
            r = 0;
            if (is_zero(dot(t, t)) && d > 0.0f) {
                r = 1;
            } else if (is_zero(d) || d < 0.0f) {
                s0 = A;
                n = 1;
                dir = AO;
            } else {
                dir = cross(cross(AB, AO), AB);
            }
        } else if (n == 2) {
            s2 = last;
            n = 3;
            r = simplex3(s0, s1, s2, n, dir);
        } else {  // doSimplex4: A = last, B = s2, C = s1, D = s0
            s3 = last;
            const V3 A = s3, B = s2, C = s1, D = s0;
            const V3 O = v3(0.0f, 0.0f, 0.0f);
            if (is_zero(point_tri_dist2(A, B, C, D))) {
                r = -1;
            } else if (is_zero(point_tri_dist2(O, A, B, C)) || is_zero(point_tri_dist2(O, A, C, D)) ||
                       is_zero(point_tri_dist2(O, A, B, D)) || is_zero(point_tri_dist2(O, B, C, D))) {
                r = 1;
            } else {
                const V3 AO = neg(A);
                const V3 AB = B - A, AC = C - A, AD = D - A;
                const V3 ABC = cross(AB, AC), ACD = cross(AC, AD), ADB = cross(AD, AB);
                const bool ab_o = signum(dot(ACD, AO)) == signum(dot(ACD, AB));
                const bool ac_o = signum(dot(ADB, AO)) == signum(dot(ADB, AC));
                const bool ad_o = signum(dot(ABC, AO)) == signum(dot(ABC, AD));
                if (ab_o && ac_o && ad_o) {
                    r = 1;
                } else {
                    if (!ab_o) {  // drop B: (D, C, A)
                        s2 = A;
                    } else if (!ac_o) {  // drop C: (B, D, A)
                        s1 = D;
                        s0 = B;
                        s2 = A;
                    } else {  // drop D: (C, B, A)
                        s0 = C;
                        s1 = B;
                        s2 = A;
                    }
                    n = 3;
                    r = simplex3(s0, s1, s2, n, dir);
                }
            }
        }
#if IKPSO_COLLIDE_STATS
        cs_count(cs, kCsGjkHit, r == 1);
#endif
        if (r == 1) return true;
        if (r == -1) return false;
        if (is_zero(dot(dir, dir))) return false;
    }
    return false;
}

// matrixToQuaternion (src/matrix_operations.cuh:78-109) of a world rotation
// (row-major r[row][col] = cells[col + 4*row]).
__device__ __forceinline__ void mat_to_quat(float r00, float r01, float r02, float r10, float r11, float r12,
                                            float r20, float r21, float r22, float q[4])
{
    const float tr = r00 + r11 + r22;
    if (tr > 0.0f) {
        const float S = (float)(__builtin_sqrt((double)tr + 1.0) * 2.0);
        q[3] = (float)(0.25 * (double)S);
        q[0] = (r21 - r12) / S;
        q[1] = (r02 - r20) / S;
        q[2] = (r10 - r01) / S;
    } else if ((r00 > r11) & (r00 > r22)) {
        const float S = (float)(__builtin_sqrt(1.0 + (double)r00 - (double)r11 - (double)r22) * 2.0);
        q[3] = (r21 - r12) / S;
        q[0] = (float)(0.25 * (double)S);
        q[1] = (r01 + r10) / S;
        q[2] = (r02 + r20) / S;
    } else if (r11 > r22) {
        const float S = (float)(__builtin_sqrt(1.0 + (double)r11 - (double)r00 - (double)r22) * 2.0);
        q[3] = (r02 - r20) / S;
        q[0] = (r01 + r10) / S;
        q[1] = (float)(0.25 * (double)S);
        q[2] = (r12 + r21) / S;
    } else {
        const float S = (float)(__builtin_sqrt(1.0 + (double)r22 - (double)r00 - (double)r11) * 2.0);
        q[3] = (r10 - r01) / S;
        q[0] = (r02 + r20) / S;
        q[1] = (r12 + r21) / S;
        q[2] = (float)(0.25 * (double)S);
    }
}

// Sphere test: can the two boxes' support points come within 1e-3?  (The
// margin also covers the rounding of the support points, ~1e-6 relative.)
__device__ __forceinline__ bool may_touch(float ax, float ay, float az, float ar, float bx, float by, float bz,
                                          float br)
{
    const float dx = ax - bx, dy = ay - by, dz = az - bz;
    const float reach = ar + br;
    const float scale_ = fabsf(ax) + fabsf(ay) + fabsf(az) + fabsf(bx) + fabsf(by) + fabsf(bz) + reach;
    const float lim = reach + 1e-3f + 1e-4f * scale_;
    return dx * dx + dy * dy + dz * dz <= lim * lim;
}
__device__ __forceinline__ bool may_touch(const Box& a, const Box& b)
{
    return may_touch(a.px, a.py, a.pz, a.radius, b.px, b.py, b.pz, b.radius);
}

// Bound on quat_gain of a node's quaternion for near_collider, which runs before
// the quaternion exists.  quat_gain(q) = max(1, sqrt(1 + 4 (|q|^2 - 1) |r|^2)),
// and matrixToQuaternion of a rotation matrix orthonormal to d gives |q|^2 within
// ~4d of 1; a node frame is a product of at most 3 x 32 fp32 plane rotations,
// orthonormal to ~1e-5, so quat_gain <= 1.0001.  1.01 covers |q|^2 up to 1.005,
// so every pair node_collides would test passes near_collider first.
constexpr float kGainBound = 1.01f;

// The inline sphere test of node k: may its node box or link box come near a
// collider?  One sphere around both boxes, centred at the link's midpoint m, per
// collider c: |m - c|^2 <= lim[k-1][c] -- a limit the host computes from the node's
// link length, the collider's radius and a bound on the chain's reach so that every
// pair node_collides would test (its may_touch with the quaternion's gain) passes
// here first (ikpso_api.cpp: parse_chain).  Three subtractions, a dot product and a
// compare per collider; no quaternion.
constexpr int kNearUnroll = 4;
__device__ __forceinline__ bool near_collider(float nx, float ny, float nz, float ex, float ey, float ez,
                                              const float* lim, const CollRec* coll, int count IKPSO_CS_PARAM)
{
    const float mx = (nx + ex) * 0.5f, my = (ny + ey) * 0.5f, mz = (nz + ez) * 0.5f;
    bool near = false;
    auto test = [&](int i) {
        const CollRec& c = coll[i];
        const float dx = mx - c.px, dy = my - c.py, dz = mz - c.pz;
        const bool n = dx * dx + dy * dy + dz * dz <= lim[i];
#if IKPSO_COLLIDE_STATS
        cs_count(cs, kCsPre, true);
        cs_count(cs, kCsPrePass, n);
#endif
        near = near || n;
    };
    // the first kNearUnroll colliders unrolled under uniform guards (a runtime loop's
    // back edge made the register allocator spill around it), the rest in a loop
#pragma unroll
    for (int i = 0; i < kNearUnroll; ++i)
        if (i < count) test(i);
    for (int i = kNearUnroll; i < count; ++i) test(i);
    return near;
}

// The same test with the first kNearUnroll colliders' centres and limits from the
// swarm kernels' LDS copy (SwarmShared::near4, q4 = node k's 16 floats): the same
// values and operations, so the same decisions.  One broadcast ds_read_b128 per
// collider instead of the scalar loads of the records and limits, whose waits the
// iteration paid on every node: collide leg 69.3 -> 66.2 ms (round 6).
__device__ __forceinline__ bool near_collider_lds(float nx, float ny, float nz, float ex, float ey, float ez,
                                                  const float* q4, const float* lim, const CollRec* coll, int count)
{
    const float mx = (nx + ex) * 0.5f, my = (ny + ey) * 0.5f, mz = (nz + ez) * 0.5f;
    bool near = false;
#pragma unroll
    for (int i = 0; i < kNearUnroll; ++i)
        if (i < count) {
            const float4 q = *(const float4*)(q4 + 4 * i);
            const float dx = mx - q.x, dy = my - q.y, dz = mz - q.z;
            near = near || (dx * dx + dy * dy + dz * dz <= q.w);
        }
    for (int i = kNearUnroll; i < count; ++i) {
        const CollRec& c = coll[i];
        const float dx = mx - c.px, dy = my - c.py, dz = mz - c.pz;
        near = near || (dx * dx + dy * dy + dz * dz <= lim[i]);
    }
    return near;
}

// FAST: the exact overlap test of two oriented boxes by separating axes (Gottschalk's
// OBB test: the 3 + 3 face axes and the 9 edge-pair axes), in place of GJK.  a, b:
// centres; A, B: axes (axis i at [3i..3i+2], unit); ea, eb: half extents.  Fixed
// work and no divergence (GJK: ~2.3 iterations at 0.56 SIMT efficiency, round 5) and
// no quaternion.  Exact in exact arithmetic; GJK's tolerance (a hit once the origin
// is within sqrt(FLT_EPSILON) of a simplex of support points) also counts boxes
// within ~3.5e-4 of touching, so the two may decide differently inside that band
// (the stated FAST tolerances: tests/test_gpu_collide.py).  The 1e-6 added to
// |R| guards near-parallel edge pairs (a degenerate cross axis then cannot separate).
__host__ __device__ __forceinline__ bool obb_overlap(const float a[3], const float A[9], const float ea[3], const float b[3],
                                            const float B[9], const float eb[3])
{
    float R[3][3], AR[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            R[i][j] = (A[3 * i] * B[3 * j] + A[3 * i + 1] * B[3 * j + 1]) + A[3 * i + 2] * B[3 * j + 2];
            AR[i][j] = fabsf(R[i][j]) + 1e-6f;
        }
    const float d0 = b[0] - a[0], d1 = b[1] - a[1], d2 = b[2] - a[2];
    float t[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) t[i] = (d0 * A[3 * i] + d1 * A[3 * i + 1]) + d2 * A[3 * i + 2];
    bool sep = false;
#pragma unroll
    for (int i = 0; i < 3; ++i)  // A's face axes
        sep = sep || fabsf(t[i]) > ea[i] + ((eb[0] * AR[i][0] + eb[1] * AR[i][1]) + eb[2] * AR[i][2]);
#pragma unroll
    for (int j = 0; j < 3; ++j)  // B's face axes
        sep = sep || fabsf((t[0] * R[0][j] + t[1] * R[1][j]) + t[2] * R[2][j]) >
                         ((ea[0] * AR[0][j] + ea[1] * AR[1][j]) + ea[2] * AR[2][j]) + eb[j];
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // edge pairs A_i x B_j
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
            const float ra = ea[i1] * AR[i2][j] + ea[i2] * AR[i1][j];
            const float rb = eb[j1] * AR[i][j2] + eb[j2] * AR[i][j1];
            sep = sep || fabsf(t[i2] * R[i1][j] - t[i1] * R[i2][j]) > ra + rb;
        }
    }
    return !sep;
}

// The collider block for one node with the separating-axis test (FAST, kFastSat):
// the node box and the link box (src/kernel.cu:104-118) oriented by the node's world
// rotation (the frame itself: matrixToQuaternion + quatRotVec of an orthonormal
// frame is the frame), against every collider box (ChainConsts::coll_box), each pair
// behind node_collides' sphere test with the gain's bound.
__device__ __forceinline__ bool node_collides_obb(float r00, float r01, float r02, float r10, float r11, float r12,
                                                  float r20, float r21, float r22, float nx, float ny, float nz,
                                                  float ex, float ey, float ez, float length, const CollRec* coll,
                                                  const float* cbox, int count)
{
    const float A[9] = {r00, r10, r20, r01, r11, r21, r02, r12, r22};  // the frame's columns
    const float pn[3] = {nx, ny, nz};
    const float pl[3] = {(nx + ex) * 0.5f, (ny + ey) * 0.5f, (nz + ez) * 0.5f};
    const float en[3] = {kGizmo * 0.5f, kGizmo * 0.5f, kGizmo * 0.5f};
    const float el[3] = {fabsf(length) * 0.5f, kGizmo * 0.125f, kGizmo * 0.125f};
    const float rn = sphere_radius(kGizmo, kGizmo, kGizmo, kGainBound);
    const float rl = sphere_radius(length, kGizmo * 0.25f, kGizmo * 0.25f, kGainBound);
    bool hit = false;
    for (int i = 0; i < count && !hit; ++i) {
        const CollRec& c = coll[i];
        const float* bx = cbox + 16 * i;
        if (may_touch(pn[0], pn[1], pn[2], rn, c.px, c.py, c.pz, c.radius))
            hit = obb_overlap(pn, A, en, bx + 12, bx, bx + 9);
        if (!hit && may_touch(pl[0], pl[1], pl[2], rl, c.px, c.py, c.pz, c.radius))
            hit = obb_overlap(pl, A, el, bx + 12, bx, bx + 9);
    }
    return hit;
}

// The collider block of calculateDistance for one node (src/kernel.cu:104-136):
// node box (GIZMO cube at the node) and link box (length x GIZMO/4 x GIZMO/4,
// centred between node and parent), both oriented by the node's world
// rotation, against every collider, in the reference's order (per collider: the
// node box, then the link box).  Out of line, called from the collider builds'
// finish() for the near nodes only.
__device__ __noinline__ bool node_collides(float r00, float r01, float r02, float r10, float r11, float r12,
                                           float r20, float r21, float r22, float nx, float ny, float nz, float ex,
                                           float ey, float ez, float length, const CollRec* coll,
                                           int count IKPSO_CS_PARAM)
{
#if IKPSO_COLLIDE_STATS
    cs_count(cs, kCsCalls, (int)__lane_id() == __builtin_ctzll(__builtin_amdgcn_read_exec()));
#endif
    float q[4], qi[4];
    mat_to_quat(r00, r01, r02, r10, r11, r12, r20, r21, r22, q);
    quat_inverse(q, qi);
    const float gain = quat_gain(q[0], q[1], q[2], q[3]);
    const Box nb{nx, ny, nz, q[0], q[1], q[2], q[3], qi[0], qi[1], qi[2], qi[3], kGizmo, kGizmo, kGizmo,
                 sphere_radius(kGizmo, kGizmo, kGizmo, gain)};
    const float lw = kGizmo * 0.25f;
    const Box lb{(nx + ex) * 0.5f, (ny + ey) * 0.5f, (nz + ez) * 0.5f, q[0], q[1], q[2], q[3], qi[0], qi[1], qi[2],
                 qi[3], length, lw, lw, sphere_radius(length, lw, lw, gain)};
    // one GJK site: pair j = (collider j / 2, node box if j even else link box)
    for (int j = 0; j < 2 * count; ++j) {
        const Box cb = box_from_record(coll[j >> 1]);
        const bool link = j & 1;
        const Box b{link ? lb.px : nb.px, link ? lb.py : nb.py, link ? lb.pz : nb.pz, nb.qx, nb.qy, nb.qz, nb.qw,
                    nb.ix, nb.iy, nb.iz, nb.iw, link ? lb.sx : nb.sx, link ? lb.sy : nb.sy, link ? lb.sz : nb.sz,
                    link ? lb.radius : nb.radius};
#if IKPSO_COLLIDE_STATS
        cs_count(cs, kCsExact, true);
        cs_count(cs, kCsExactPass, may_touch(b, cb));
#endif
        if (may_touch(b, cb) && gjk_intersect(b, cb IKPSO_CS_ARG)) return true;
    }
    return false;
}

#pragma clang fp contract(fast)  // the HIP default (-ffp-contract=fast-honor-pragmas)

}  // namespace ikpso
