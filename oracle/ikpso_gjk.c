/*
 * ikpso_gjk.c -- CPU restatement of the reference's collider term of the
 * fitness (box-box GJK intersection test).  TEST INFRASTRUCTURE ONLY, like
 * ikpso_oracle.c: the parity checker for the device collision code, never
 * linked into the product.
 *
 * Reference (src/ = InverseKinematicsResearch/InverseKinematicsResearch/):
 *   calculateDistance collider block  src/kernel.cu:104-136 -> orc_node_collides()
 *   matrixToQuaternion                src/matrix_operations.cuh:78-109 -> mat_to_quat()
 *   supportBox / SupportCalc / firstDir src/kernel.cu:499-530,594-612 -> support_box(), support_calc()
 *   GJKIntersect / GJK                src/kernel.cu:532-592 -> orc_gjk_intersect()
 *   doSimplex / doSimplex2/3/4        src/kernel.cu:614-870 -> simplex2/3/4()
 *   Vec3PointTriDist2 / PointSegmentDist src/kernel.cu:872-1010 -> point_tri_dist2(), point_seg_dist2()
 *   quatRotVec / quatInvert(2)        src/kernel.cu:1012-1061 -> quat_rot(), quat_inv()
 *   Signum / tripleCross / IsZERO     src/kernel.cu:1063-1100
 *   obj_t                             src/BoxCollider.h:4-10 -> orc_box (x, y, z are full edge lengths)
 *   GJK_ITERATIONS = 50, GIZMO_SIZE = 0.2f  src/ik_constants.h
 * The reference's GJK is itself a port of libccd's GJK (ccd_gjk / __ccdGJK,
 * libccd 2.x, BSD): not vendored as a library, its arithmetic is the code
 * above, which this file follows operation for operation (fp32, no FMA
 * contraction, -ffp-contract=off; matrixToQuaternion's sqrt in double as the
 * reference's `sqrt(tr + 1.0)` promotes).
 *
 * Semantics: the fitness is FLT_MAX when any node box (GIZMO_SIZE cube at the
 * node, oriented by the node frame) or link box (length x GIZMO/4 x GIZMO/4,
 * centred between the node and its parent, oriented by the node frame) of the
 * particle intersects any collider; otherwise it is unchanged.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

/* obj_t (src/BoxCollider.h:4-10): 48 bytes, quat float4-aligned. */
typedef struct {
    float x, y, z;
    float pos[3];
    float pad_[2];
    float quat[4]; /* x, y, z, w */
} orc_box;

int orc_sizeof_box(void) { return (int)sizeof(orc_box); }

typedef struct { float x, y, z; } v3;

static v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 vscale(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
/* float3Dot: ((x*x') + y*y') + z*z' */
static float vdot(v3 a, v3 b)
{
    float d = a.x * b.x;
    d += a.y * b.y;
    d += a.z * b.z;
    return d;
}
static v3 vcross(v3 a, v3 b)
{
    return mk((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x));
}
static float vlen2(v3 a) { return vdot(a, a); } /* float3Len is the SQUARED length */
static int veq(v3 a, v3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

static float fabs_ref(float v) { return v > 0 ? v : -v; }
static int is_zero(float v) { return fabs_ref(v) < FLT_EPSILON; }
static int sgn(float v) { return is_zero(v) ? 0 : (v < 0.0f ? -1 : 1); }
/* tripleCross(a, b, c) = (a x b) x c */
static v3 triple(v3 a, v3 b, v3 c) { return vcross(vcross(a, b), c); }

/* quatRotVec: v + 2 * cross(q.xyz, cross(q.xyz, v) + q.w * v), in the
 * reference's expanded form and order (src/kernel.cu:1012-1037). */
static v3 quat_rot(v3 v, const float q[4])
{
    const float x = q[0], y = q[1], z = q[2], w = q[3];
    const float c1x = y * v.z - z * v.y + w * v.x;
    const float c1y = z * v.x - x * v.z + w * v.y;
    const float c1z = x * v.y - y * v.x + w * v.z;
    const float c2x = y * c1z - z * c1y;
    const float c2y = z * c1x - x * c1z;
    const float c2z = x * c1y - y * c1x;
    return mk(v.x + 2.0f * c2x, v.y + 2.0f * c2y, v.z + 2.0f * c2z);
}

/* quatInvert2: copy, then conjugate / |q|^2 unless |q|^2 < FLT_EPSILON (copy kept). */
static void quat_inv(const float q[4], float out[4])
{
    memcpy(out, q, sizeof(float) * 4);
    float l2 = ((q[0] * q[0]) + (q[1] * q[1]) + (q[2] * q[2])) + (q[3] * q[3]);
    if (l2 < FLT_EPSILON) return;
    l2 = 1.0f / l2;
    out[0] = -q[0] * l2;
    out[1] = -q[1] * l2;
    out[2] = -q[2] * l2;
    out[3] = q[3] * l2;
}

/* supportBox: rotate the direction into the box frame, take the signed
 * half-extent per axis (0 where the direction component IsZERO), rotate back, add
 * the centre. */
static v3 support_box(const orc_box* b, v3 dir)
{
    float qi[4];
    quat_inv(b->quat, qi);
    const v3 d = quat_rot(dir, qi);
    v3 v = mk((float)sgn(d.x) * b->x * 0.5f, (float)sgn(d.y) * b->y * 0.5f, (float)sgn(d.z) * b->z * 0.5f);
    v = quat_rot(v, b->quat);
    return vadd(v, mk(b->pos[0], b->pos[1], b->pos[2]));
}

/* SupportCalc: point of the Minkowski difference A - B furthest along dir. */
static v3 support_calc(const orc_box* a, const orc_box* b, v3 dir)
{
    const v3 v1 = support_box(a, dir);
    const v3 v2 = support_box(b, vscale(dir, -1.0f));
    return vsub(v1, v2);
}

/* PointSegmentDist (src/kernel.cu:955-1010); `want_witness` selects the
 * reference's witness branch, whose arithmetic differs from the plain one. */
static float point_seg_dist2(v3 P, v3 x0, v3 b, int want_witness)
{
    const v3 d = vsub(b, x0);
    const v3 a = vsub(x0, P);
    float t = -1.0f * vdot(a, d);
    t /= vlen2(d);
    if (t < 0.0f || is_zero(t)) return vlen2(vsub(x0, P));
    if (t > 1.0f || t == 1.0f) return vlen2(vsub(b, P));
    if (want_witness) {
        const v3 w = vadd(vscale(d, t), x0);
        return vlen2(vsub(w, P));
    }
    return vlen2(vadd(vscale(d, t), a));
}

/* Vec3PointTriDist2 with witness == NULL (the only way GJK calls it). */
static float point_tri_dist2(v3 P, v3 x0, v3 B, v3 C)
{
    const v3 d1 = vsub(B, x0), d2 = vsub(C, x0), a = vsub(x0, P);
    const float u = vdot(a, a), v = vdot(d1, d1), w = vdot(d2, d2);
    const float p = vdot(a, d1), q = vdot(a, d2), r = vdot(d1, d2);
    const float den = w * v - r * r;
    float s, t;
    if (is_zero(den)) {
        s = t = -1.0f;
    } else {
        s = (q * r - w * p) / den;
        t = (-s * r - q) / w;
    }
    if ((is_zero(s) || s > 0.0f) && (s == 1.0f || s < 1.0f) && (is_zero(t) || t > 0.0f) &&
        (t == 1.0f || t < 1.0f) && (t + s == 1.0f || t + s < 1.0f)) {
        float dist = s * s * v;
        dist += t * t * w;
        dist += 2.0f * s * t * r;
        dist += 2.0f * s * p;
        dist += 2.0f * t * q;
        dist += u;
        return dist;
    }
    float dist = point_seg_dist2(P, x0, B, 0);
    float d2b = point_seg_dist2(P, x0, C, 1);
    if (d2b < dist) dist = d2b;
    d2b = point_seg_dist2(P, B, C, 1);
    if (d2b < dist) dist = d2b;
    return dist;
}

/* The simplex: pts[0..n-1], the newest point last (simplex_t, src/simplex.cuh). */
typedef struct {
    v3 pts[4];
    int n;
} simplex;

/* doSimplex2 (src/kernel.cu:631-672) */
static int simplex2(simplex* s, v3* dir)
{
    const v3 A = s->pts[s->n - 1], B = s->pts[0];
    const v3 AB = vsub(B, A), AO = vscale(A, -1.0f);
    const float dot = vdot(AB, AO);
    const v3 tmp = vcross(AB, AO);
    if (is_zero(vlen2(tmp)) && dot > 0.0f) return 1;
    if (is_zero(dot) || dot < 0.0f) {
        s->pts[0] = A;
        s->n = 1;
        *dir = AO;
    } else {
        *dir = triple(AB, AO, AB);
    }
    return 0;
}

/* doSimplex3 (src/kernel.cu:674-770) */
static int simplex3(simplex* s, v3* dir)
{
    const v3 O = mk(0.0f, 0.0f, 0.0f);
    const v3 A = s->pts[s->n - 1], B = s->pts[1], C = s->pts[0];
    if (is_zero(point_tri_dist2(O, A, B, C))) return 1;
    if (veq(A, B) || veq(A, C)) return -1;
    const v3 AO = vscale(A, -1.0f);
    const v3 AB = vsub(B, A), AC = vsub(C, A);
    const v3 ABC = vcross(AB, AC);
    float dot = vdot(vcross(ABC, AC), AO);
    if (is_zero(dot) || dot > 0.0f) {
        dot = vdot(AC, AO);
        if (is_zero(dot) || dot > 0.0f) {
            s->pts[1] = A; /* C stays at 0 */
            s->n = 2;
            *dir = triple(AC, AO, AC);
        } else {
            dot = vdot(AB, AO);
            if (is_zero(dot) || dot > 0.0f) {
                s->pts[0] = B;
                s->pts[1] = A;
                s->n = 2;
                *dir = triple(AB, AO, AB);
            } else {
                s->pts[0] = A;
                s->n = 1;
                *dir = AO;
            }
        }
    } else {
        dot = vdot(vcross(AB, ABC), AO);
        if (is_zero(dot) || dot > 0.0f) {
            dot = vdot(AB, AO);
            if (is_zero(dot) || dot > 0.0f) {
                s->pts[0] = B;
                s->pts[1] = A;
                s->n = 2;
                *dir = triple(AB, AO, AB);
            } else {
                s->pts[0] = A;
                s->n = 1;
                *dir = AO;
            }
        } else {
            dot = vdot(ABC, AO);
            if (is_zero(dot) || dot > 0.0f) {
                *dir = ABC;
            } else {
                /* swap B and C, keep the size (3) */
                s->pts[0] = B;
                s->pts[1] = C;
                *dir = vscale(ABC, -1.0f);
            }
        }
    }
    return 0;
}

/* doSimplex4 (src/kernel.cu:772-870) */
static int simplex4(simplex* s, v3* dir)
{
    const v3 O = mk(0.0f, 0.0f, 0.0f);
    const v3 A = s->pts[3], B = s->pts[2], C = s->pts[1], D = s->pts[0];
    if (is_zero(point_tri_dist2(A, B, C, D))) return -1;
    if (is_zero(point_tri_dist2(O, A, B, C))) return 1;
    if (is_zero(point_tri_dist2(O, A, C, D))) return 1;
    if (is_zero(point_tri_dist2(O, A, B, D))) return 1;
    if (is_zero(point_tri_dist2(O, B, C, D))) return 1;
    const v3 AO = vscale(A, -1.0f);
    const v3 AB = vsub(B, A), AC = vsub(C, A), AD = vsub(D, A);
    const v3 ABC = vcross(AB, AC), ACD = vcross(AC, AD), ADB = vcross(AD, AB);
    const int b_on_acd = sgn(vdot(ACD, AB));
    const int c_on_adb = sgn(vdot(ADB, AC));
    const int d_on_abc = sgn(vdot(ABC, AD));
    const int ab_o = sgn(vdot(ACD, AO)) == b_on_acd;
    const int ac_o = sgn(vdot(ADB, AO)) == c_on_adb;
    const int ad_o = sgn(vdot(ABC, AO)) == d_on_abc;
    if (ab_o && ac_o && ad_o) return 1;
    if (!ab_o) {
        s->pts[2] = A; /* drop B */
    } else if (!ac_o) {
        s->pts[1] = D; /* drop C */
        s->pts[0] = B;
        s->pts[2] = A;
    } else {
        s->pts[0] = C; /* drop D */
        s->pts[1] = B;
        s->pts[2] = A;
    }
    s->n = 3;
    return simplex3(s, dir);
}

#define ORC_GJK_ITERATIONS 50 /* GJK_ITERATIONS, src/ik_constants.h */

/* GJKIntersect (src/kernel.cu:532-592): 1 if the boxes intersect. */
int orc_gjk_intersect(const orc_box* a, const orc_box* b)
{
    simplex s;
    v3 dir = mk(1.0f, 1.0f, 0.0f); /* firstDir */
    v3 last = support_calc(a, b, dir);
    s.pts[0] = last;
    s.n = 1;
    dir = vscale(last, -1.0f);
    for (int it = 0; it < ORC_GJK_ITERATIONS; it++) {
        last = support_calc(a, b, dir);
        if (vdot(last, dir) < 0.0f) return 0;
        s.pts[s.n++] = last;
        int r;
        if (s.n == 2)
            r = simplex2(&s, &dir);
        else if (s.n == 3)
            r = simplex3(&s, &dir);
        else
            r = simplex4(&s, &dir);
        if (r == 1) return 1;
        if (r == -1) return 0;
        if (is_zero(vlen2(dir))) return 0;
    }
    return 0;
}

/* matrixToQuaternion (src/matrix_operations.cuh:78-109) of a row-major 4x4
 * (cells[col + 4*row]); the sqrt argument and product are evaluated in double. */
static void mat_to_quat(const float* m, float q[4])
{
    const float tr = m[0] + m[5] + m[10];
    float S;
    if (tr > 0) {
        S = (float)(sqrt((double)tr + 1.0) * 2);
        q[3] = (float)(0.25 * (double)S);
        q[0] = (m[9] - m[6]) / S;
        q[1] = (m[2] - m[8]) / S;
        q[2] = (m[4] - m[1]) / S;
    } else if ((m[0] > m[5]) & (m[0] > m[10])) {
        S = (float)(sqrt(1.0 + (double)m[0] - (double)m[5] - (double)m[10]) * 2);
        q[3] = (m[9] - m[6]) / S;
        q[0] = (float)(0.25 * (double)S);
        q[1] = (m[1] + m[4]) / S;
        q[2] = (m[2] + m[8]) / S;
    } else if (m[5] > m[10]) {
        S = (float)(sqrt(1.0 + (double)m[5] - (double)m[0] - (double)m[10]) * 2);
        q[3] = (m[2] - m[8]) / S;
        q[0] = (m[1] + m[4]) / S;
        q[1] = (float)(0.25 * (double)S);
        q[2] = (m[6] + m[9]) / S;
    } else {
        S = (float)(sqrt(1.0 + (double)m[10] - (double)m[0] - (double)m[5]) * 2);
        q[3] = (m[4] - m[1]) / S;
        q[0] = (m[2] + m[8]) / S;
        q[1] = (m[6] + m[9]) / S;
        q[2] = (float)(0.25 * (double)S);
    }
}

#define ORC_GIZMO 0.2f /* GIZMO_SIZE, src/ik_constants.h */

/* The collider block of calculateDistance for node `ind` (src/kernel.cu:104-136):
 * `node` = the node's world matrix, `parent` = its parent's. */
int orc_node_collides(const float* node, const float* parent, float length, const orc_box* colliders, int count)
{
    if (count <= 0) return 0;
    /* multiplyMatByVec(model, (0,0,0,1)): exact picks of the translation column */
    const float sx = node[3], sy = node[7], sz = node[11], sw = node[15];
    const float ex = parent[3], ey = parent[7], ez = parent[11], ew = parent[15];
    float q[4];
    mat_to_quat(node, q);
    orc_box nb, lb;
    memset(&nb, 0, sizeof(nb));
    memset(&lb, 0, sizeof(lb));
    nb.pos[0] = sx;
    nb.pos[1] = sy;
    nb.pos[2] = sz;
    memcpy(nb.quat, q, sizeof(q));
    nb.x = nb.y = nb.z = ORC_GIZMO;
    /* centerPos = (startPos + endPos) * 0.5f (float4 ops; w unused) */
    (void)sw;
    (void)ew;
    lb.pos[0] = (sx + ex) * 0.5f;
    lb.pos[1] = (sy + ey) * 0.5f;
    lb.pos[2] = (sz + ez) * 0.5f;
    memcpy(lb.quat, q, sizeof(q));
    lb.x = length;
    lb.y = lb.z = ORC_GIZMO * 0.25f;
    for (int i = 0; i < count; i++) {
        if (orc_gjk_intersect(&nb, &colliders[i])) return 1;
        if (orc_gjk_intersect(&lb, &colliders[i])) return 1;
    }
    return 0;
}
