// ikpso_device.h -- device building blocks of the MI355X PSO-IK hot path.
//
// Everything here is written for gfx950 (CDNA4, wave64).  Reference being
// replaced (src/ = InverseKinematicsResearch/InverseKinematicsResearch/):
//   XORWOW generator            curand_init/curand_uniform used at src/utility_kernels.cuh:28,
//                               src/kernel.cu:164-166,261
//   forward kinematics          updateChainMatrices src/kernel.cu:31-62 + src/matrix_operations.cuh
//   fitness                     calculateDistance src/kernel.cu:64-151 (collider block: ikpso_collide.h)
//   velocity/position update    simulateParticlesKernel src/kernel.cu:153-189
//   swarm argmin                thrust::min_element src/kernel.cu:297,315 (first minimum)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ikpso_collide.h"
#include "ikpso_params.h"

// gfx950 VALU issue costs (tools/probes/valu_probe.hip, 4 waves per SIMD):
// a wave64 v_add_u32 / v_xor_b32 / v_bitop3_b32 / v_fma_f32 on VGPR, inline or
// literal operands issues every ~2.1-2.5 cycles per SIMD, but every
// v_lshlrev_b32 and every VALU op that reads an SGPR takes ~4.1.  So the
// generator's t << 1 is issued as t + t.  (Holding the sincos sign mask or the
// PSO coefficients in VGPRs instead of SGPRs measured no better: DESIGN.md.)

namespace ikpso {

// ------------------------------------------------------------ bit helpers
// gfx950 v_bitop3_b32: any 3-input bitwise function in one instruction (LUT
// over a = 0xF0, b = 0xCC, c = 0xAA).  Host builds (unit tests) use the plain
// expression.
__host__ __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}

// t << 1 as t + t (v_add_u32 issues twice as fast as v_lshlrev_b32; opaque to
// the compiler, which would canonicalise an add back into the shift).
__host__ __device__ __forceinline__ uint32_t shl1(uint32_t t)
{
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(t));
    return r;
#else
    return t << 1;
#endif
}

// a ^ (b & 0x80000000): flip the sign of the float bits a where b's top bit is set.
__host__ __device__ __forceinline__ uint32_t xor_sign(uint32_t a, uint32_t b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, 0x80000000u, 0x78);
#else
    return a ^ (b & 0x80000000u);
#endif
}

__host__ __device__ __forceinline__ float as_float(uint32_t u)
{
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}
__host__ __device__ __forceinline__ uint32_t as_uint(float f)
{
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    return u;
}

// ---------------------------------------------------------------- XORWOW
// cuRAND XORWOW restated: state {d, v[5]}; curand() and curand_uniform().
// kAddShl: issue t << 1 as t + t (shl1; same bits).
template <bool kAddShl>
struct XorwowT {
    uint32_t d, v0, v1, v2, v3, v4;

    __host__ __device__ __forceinline__ uint32_t next()
    {
        const uint32_t t = v0 ^ (v0 >> 2);
        v0 = v1;
        v1 = v2;
        v2 = v3;
        v3 = v4;
        v4 = xor3(v4, v4 << 4, t) ^ (kAddShl ? shl1(t) : t << 1);  // (v4 ^ (v4 << 4)) ^ (t ^ (t << 1))
        d += 362437u;
        return v4 + d;  // (fused into v_add3_u32 v4 + d_old + 362437; two opaque 2-cycle adds measured 4 % slower)
    }
    // x * 2^-32 + 2^-33 in (0, 1]; the product is exact, so fused or not the
    // result is the same single rounding.
    __host__ __device__ __forceinline__ float uniform()
    {
        return __builtin_fmaf((float)next(), 2.3283064e-10f, 1.16415322e-10f);
    }
    // c * uniform() with the scale folded in: fma(x, c*2^-32, c*2^-33).
    __host__ __device__ __forceinline__ float scaled(float q, float h)
    {
        return __builtin_fmaf((float)next(), q, h);
    }
};
using Xorwow = XorwowT<false>;

__host__ __device__ inline void xorwow_seed(uint64_t seed, uint32_t st[6])
{
    const uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    const uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0;
    const uint32_t t1 = 2591861531u * s1;
    st[0] = 6615241u + t1 + t0;
    st[1] = 123456789u + t0;
    st[2] = 362436069u ^ t0;
    st[3] = 521288629u + t1;
    st[4] = 88675123u ^ t1;
    st[5] = 5783321u + t0;
}

// ------------------------------------------------------------------ sincos
// The particle angles are clamped to the joint limits, so |x| is small; the
// library sincosf inlines a Payne-Hanek path for huge arguments at every call
// site (42 sites per particle-update), which costs ~12k instructions of code
// and spills the particle state.  Both variants below reduce by pi/2 inline
// and are accurate for |x| < 2^12 rad.

// FAST: Cody-Waite reduction by pi/2 in two FMA steps (exact enough for
// |x| < 2^12), minimax polynomials on [-pi/4, pi/4] (sin odd degree 7, cos
// Horner in z = r^2), quadrant fix-up by one select pair and two bitop3 sign
// flips.  Measured on gfx950 against correctly rounded sin/cos over 2^26
// arguments in [-100, 100]: 71-73% correctly rounded (tools/probes/trig_probe.hip);
// exhaustively over every float |x| < 4096: max 2 ulp, 7.2e-8 abs.
// TRIG 1 (kTrigHw): the transcendental unit instead (below); TRIG 2 (kTrigHwRev):
// the same with the angle given in revolutions (kTermRev kernels), so the
// conversion multiply disappears.
// TRIG 3 (kTrigPolyRev): the polynomial on an angle in revolutions (x * 2pi first; only
// the IKPSO_FAST_HW_TRIG=0 attribution builds).
constexpr int kTrigPoly = 0, kTrigHw = 1, kTrigHwRev = 2, kTrigPolyRev = 3;
template <int HW = kTrigPoly>
__host__ __device__ __forceinline__ void sincos_fast(float x, float* s_out, float* c_out)
{
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (HW == kTrigHwRev) {
        *s_out = __builtin_amdgcn_sinf(x);
        *c_out = __builtin_amdgcn_cosf(x);
        return;
    }
    if constexpr (HW == kTrigHw) {
        // v_sin_f32 / v_cos_f32 on x / 2pi (revolutions; the transcendental unit
        // reduces its own argument).  tools/probes/trig_probe.hip on gfx950: max
        // abs error 4.8e-7 on [0, 2pi] and 2.7e-7 on [-pi, pi] (vs 6e-8 for the
        // polynomial); 8 cycles per wave64 op each (tools/probes/valu_probe.hip),
        // 3 instructions per angle against ~20 for the polynomial: -7 % kernel
        // time on the reference scene, -9 % on the 2-wave D = 60 cooperative
        // kernel once its loop stopped spilling (it was +13 % before).
        // x / 2pi with the constant in two parts: fl(1 / 2pi) = 0.15915494f is 4.0e-8
        // (relative) short of 1 / 2pi, so x * 0.15915494f turns every joint by that
        // fraction less than x -- a bias the optimiser answers with larger angles, which
        // the angle term then prices (round 6: the collider builds' strict tier-B count
        // 133 worse / 91 better).  The low part's FMA rounds the product once, unbiased.
        const float rev = __builtin_fmaf(x, 6.42063833e-9f, x * 0.159154936671257019f);
        *s_out = __builtin_amdgcn_sinf(rev);
        *c_out = __builtin_amdgcn_cosf(rev);
        return;
    }
#endif
    if constexpr (HW == kTrigPolyRev) x = x * 6.28318530717958648f;
    // Quadrant by the round-to-integer magic constant: k_big = x*2/pi + 1.5*2^23
    // holds q = rint(x*2/pi) in its low mantissa bits (one FMA instead of a
    // multiply, a rint and a float->int conversion); the swap of sin and cos
    // by a bitfield-extended mask and two bitop3 selects.
    const float kb = __builtin_fmaf(x, 0.636619772367581343f, 12582912.0f);
    const float k = kb - 12582912.0f;
    const uint32_t qb = as_uint(kb);
    float r = __builtin_fmaf(-k, 1.57079637050628662109375f, x);
    r = __builtin_fmaf(-k, -4.37113900018624283e-8f, r);
    const float z = r * r;
    const float sp = __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    const float sv = __builtin_fmaf(sp * z, r, r);
    float cp = __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                              4.166664568298827e-2f);
    cp = __builtin_fmaf(cp, z, -0.5f);
    const float cv = __builtin_fmaf(cp, z, 1.0f);
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)qb, 0, 1);  // q odd: all ones
    const uint32_t s1 = __builtin_amdgcn_bitop3_b32(m, as_uint(cv), as_uint(sv), 0xCA);  // m ? cv : sv
    const uint32_t c1 = __builtin_amdgcn_bitop3_b32(m, as_uint(sv), as_uint(cv), 0xCA);  // m ? sv : cv
#else
    const uint32_t m = (qb & 1u) ? 0xFFFFFFFFu : 0u;
    const uint32_t s1 = (m & as_uint(cv)) | (~m & as_uint(sv));
    const uint32_t c1 = (m & as_uint(sv)) | (~m & as_uint(cv));
#endif
    const uint32_t t = qb << 30;  // bit 31: q & 2 (sin sign); (q + 1) & 2 for cos
    *s_out = as_float(xor_sign(s1, t));
    *c_out = as_float(xor_sign(c1, t + 0x40000000u));
}

// REFERENCE: the reduction and the polynomials (fdlibm __kernel_sin /
// __kernel_cos coefficients) in fp64, rounded once to fp32.  Equal, bit for bit,
// to the CPU oracle's (float)sin((double)x) / (float)cos((double)x) on EVERY
// float with |x| < 4096 (both signs, zeros and subnormals included): checked
// exhaustively on the host, tests/test_sincos_exhaustive.py.
//   * the quadrant by the fp64 round-to-integer magic constant (k = rint(x*2/pi):
//     one fma and one add instead of a multiply, a rint and two conversions);
//     near a quadrant boundary k may differ by one from the fp32 rint's, the
//     reduced argument then lies just past pi/4, where the polynomials are as
//     accurate;
//   * sin(r) = r * (1 + z*S(z)): the product keeps the sign of r = -0 (the
//     fma(r*z, S, r) form returned +0 for sin(-0), the one float on which it
//     differed from the oracle), at the same operation count;
//   * the quadrant's swap and signs as bit selects on the fp32 results (bitop3 /
//     xor instead of compares and cndmasks).
__host__ __device__ __forceinline__ void sincos_reference(float x, float* s_out, float* c_out)
{
    const double xd = (double)x;
    const double kb = __builtin_fma(xd, 6.36619772367581382433e-01, 6755399441055744.0);  // 1.5 * 2^52 + k
    const double k = kb - 6755399441055744.0;
    uint64_t kbits;
    __builtin_memcpy(&kbits, &kb, 8);
    const uint32_t q = (uint32_t)kbits;  // k mod 2^32 (two's complement)
    double r = __builtin_fma(-k, 1.57079632673412561417e+00, xd);
    r = __builtin_fma(-k, 6.07710050650619224932e-11, r);
    const double z = r * r;
    double sp = __builtin_fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);
    sp = __builtin_fma(z, sp, 2.75573137070700676789e-06);
    sp = __builtin_fma(z, sp, -1.98412698298579493134e-04);
    sp = __builtin_fma(z, sp, 8.33333333332248946124e-03);
    sp = __builtin_fma(z, sp, -1.66666666666666324348e-01);
    const double sv = r * __builtin_fma(z, sp, 1.0);
    double cp = __builtin_fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);
    cp = __builtin_fma(z, cp, -2.75573143513906633035e-07);
    cp = __builtin_fma(z, cp, 2.48015872894767294178e-05);
    cp = __builtin_fma(z, cp, -1.38888888888741095749e-03);
    cp = __builtin_fma(z, cp, 4.16666666666666019037e-02);
    const double cv = __builtin_fma(z * z, cp, __builtin_fma(-0.5, z, 1.0));
    const uint32_t sf = as_uint((float)sv), cf = as_uint((float)cv);
    const uint32_t m = 0u - (q & 1u);  // q odd: all ones (swap)
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t s1 = __builtin_amdgcn_bitop3_b32(m, cf, sf, 0xCA);  // m ? cf : sf
    const uint32_t c1 = __builtin_amdgcn_bitop3_b32(m, sf, cf, 0xCA);  // m ? sf : cf
#else
    const uint32_t s1 = (m & cf) | (~m & sf);
    const uint32_t c1 = (m & sf) | (~m & cf);
#endif
    const uint32_t t = q << 30;  // bit 31: q & 2 (sin sign); (q + 1) & 2 for cos
    *s_out = as_float(xor_sign(s1, t));
    *c_out = as_float(xor_sign(c1, t + 0x40000000u));
}

// ------------------------------------------------------------- topologies
// The kinematic tree is a compile-time parameter so that every node frame
// lives in registers (a runtime-indexed frame array would go to scratch) and
// the per-node effector test is resolved at compile time.  parent(k) and
// effector(k) for k = 1..J; node 0 is the origin.

// The reference's scene (src/Main.cpp:76-116): origin -> 4 elbows -> 3 wrist
// effectors hanging off the last elbow; DFS parent indices [-1,0,1,2,3,4,4,4].
//   A: angles per node (3 Euler angles; 1 for the folded chain), D = A*J the
//   kernel's dimensions; kDH: the folded serial chain (FitnessAccDH).
struct TopoRef7 {
    static constexpr int J = 7, A = 3, D = 21;
    static constexpr bool kGeneric = false, kDH = false;
    __host__ __device__ static constexpr int parent(int k) { return k <= 5 ? k - 1 : 4; }
    __host__ __device__ static constexpr bool leaf(int k) { return k >= 5; }  // no child reads its frame
    __host__ __device__ static constexpr bool effector(int k) { return k >= 5; }
};

// Serial chain of J joints with one tip effector (BASELINE config 5: J = 20).
template <int J_>
struct TopoSerialTip {
    static constexpr int J = J_, A = 3, D = 3 * J_;
    static constexpr bool kGeneric = false, kDH = false;
    __host__ __device__ static constexpr int parent(int k) { return k - 1; }
    __host__ __device__ static constexpr bool leaf(int k) { return k == J_; }
    __host__ __device__ static constexpr bool effector(int k) { return k == J_; }
};

// Any tree with J joints: parent indices read at run time (frames in scratch),
// every node weighted by its effector weight (0 for non-effectors).
template <int J_>
struct TopoGeneric {
    static constexpr int J = J_, A = 3, D = 3 * J_;
    static constexpr bool kGeneric = true, kDH = false;
    __host__ __device__ static constexpr int parent(int k) { return k - 1; }  // unused
    __host__ __device__ static constexpr bool leaf(int) { return false; }
    __host__ __device__ static constexpr bool effector(int) { return true; }
};

// A serial chain with a tip effector whose free angles are folded into J
// single-axis joints (extension, SURVEY.md §8(f) row 4: joint-axis mask / DH
// arms): every free Euler axis c of node k is written R_c(t) = Q_c Rz(t) Q_c^T,
// and every constant factor between two free axes -- the locked Euler angles,
// the Q_c, whole locked nodes, the origin transform -- is multiplied out on the
// host (fp64) into C_j, and every link length into the offset s_j:
//   W_j = W_{j-1} C_j Rz(t_j),   q_j = q_{j-1} + W_j s_j,   tip = q_J.
// One sincos per free angle and no work for locked ones (the Euler form pays 3
// sincos per node and, with locked axes emulated by equal clamp bounds, draws
// and updates for every dead dimension).  FAST arithmetic only: REFERENCE runs
// use the Euler kernels with the mask, which keep the reference's operation
// order.  J = number of free angles = D.
template <int J_>
struct TopoDH {
    static constexpr int J = J_, A = 1, D = J_;
    static constexpr bool kGeneric = false, kDH = true;
    __host__ __device__ static constexpr int parent(int k) { return k - 1; }
    __host__ __device__ static constexpr bool leaf(int k) { return k == J_; }
    __host__ __device__ static constexpr bool effector(int k) { return k == J_; }
};

// Free-dimension helpers (ChainConsts::free_mask, identity without a mask).
template <class CC>
__device__ __forceinline__ bool dim_free(const CC& cc, int d)
{
    return (cc.free_mask >> d) & 1;
}
template <class CC>
__device__ __forceinline__ int dim_rank(const CC& cc, int d)  // index among the free dimensions
{
    return __builtin_popcountll(cc.free_mask & ((1ull << d) - 1));
}

// ------------------------------------------------------------------ frames
// World transform of one node: rotation R (row-major 3x3) and position p.
struct Frame {
    float r00, r01, r02, r10, r11, r12, r20, r21, r22;
    float px, py, pz;
};

__device__ __forceinline__ Frame origin_frame(const float* m0)
{
    Frame f;
    f.r00 = m0[0]; f.r01 = m0[1]; f.r02 = m0[2];  f.px = m0[3];
    f.r10 = m0[4]; f.r11 = m0[5]; f.r12 = m0[6];  f.py = m0[7];
    f.r20 = m0[8]; f.r21 = m0[9]; f.r22 = m0[10]; f.pz = m0[11];
    return f;
}

// FAST: closed-form local rotation Rx(a)Ry(b)Rz(c), then world = parent * local,
// FMA contraction allowed.  For leaf nodes only the position is consumed and
// the compiler drops the unused rotation entries.
// Sines and cosines of a node's A angles, computed ahead of the node's FK
// (FAST: swarm_step evaluates them one node early so the transcendental
// latency hides under the previous node's FK).
template <int A>
struct NodeTrig {
    float s[A], c[A];
};

template <int HW, int A>
__device__ __forceinline__ NodeTrig<A> node_trig(const float* ang)
{
    NodeTrig<A> t;
#pragma unroll
    for (int ax = 0; ax < A; ++ax) sincos_fast<HW>(ang[ax], &t.s[ax], &t.c[ax]);
    return t;
}

__device__ __forceinline__ Frame child_frame_fast_sc(const Frame& P, float sa, float ca, float sb, float cb, float sc,
                                                     float cc, float len)
{
    const float p = sa * sb, q = ca * sb;
    const float l00 = cb * cc, l01 = -cb * sc, l02 = sb;
    const float l10 = p * cc + ca * sc, l11 = ca * cc - p * sc, l12 = -sa * cb;
    const float l20 = sa * sc - q * cc, l21 = q * sc + sa * cc, l22 = ca * cb;
    Frame W;
    W.r00 = P.r00 * l00 + P.r01 * l10 + P.r02 * l20;
    W.r01 = P.r00 * l01 + P.r01 * l11 + P.r02 * l21;
    W.r02 = P.r00 * l02 + P.r01 * l12 + P.r02 * l22;
    W.r10 = P.r10 * l00 + P.r11 * l10 + P.r12 * l20;
    W.r11 = P.r10 * l01 + P.r11 * l11 + P.r12 * l21;
    W.r12 = P.r10 * l02 + P.r11 * l12 + P.r12 * l22;
    W.r20 = P.r20 * l00 + P.r21 * l10 + P.r22 * l20;
    W.r21 = P.r20 * l01 + P.r21 * l11 + P.r22 * l21;
    W.r22 = P.r20 * l02 + P.r21 * l12 + P.r22 * l22;
    W.px = P.px + len * W.r00;
    W.py = P.py + len * W.r10;
    W.pz = P.pz + len * W.r20;
    return W;
}

template <int HW>
__device__ __forceinline__ Frame child_frame_fast(const Frame& P, float a, float b, float c, float len)
{
    float sa, ca, sb, cb, sc, cc;
    sincos_fast<HW>(a, &sa, &ca);
    sincos_fast<HW>(b, &sb, &cb);
    sincos_fast<HW>(c, &sc, &cc);
    return child_frame_fast_sc(P, sa, ca, sb, cb, sc, cc, len);
}

// FAST, interior nodes (the whole world rotation is consumed by the children):
// apply Rx, Ry, Rz to the parent's columns in turn -- each is a plane rotation
// of two columns (12 multiply-adds), 36 in all against 14 + 27 for building
// the local matrix and multiplying it in.  Leaves, which only need the first
// column, keep the closed form (the compiler then drops the other columns).
__device__ __forceinline__ Frame child_frame_fast_seq_sc(const Frame& P, float sa, float ca, float sb, float cb,
                                                         float sc, float cc, float len)
{
    // * Rx(a): columns 1, 2 become (ca c1 + sa c2, ca c2 - sa c1)
    const float x01 = P.r01 * ca + P.r02 * sa, x02 = P.r02 * ca - P.r01 * sa;
    const float x11 = P.r11 * ca + P.r12 * sa, x12 = P.r12 * ca - P.r11 * sa;
    const float x21 = P.r21 * ca + P.r22 * sa, x22 = P.r22 * ca - P.r21 * sa;
    // * Ry(b): columns 0, 2 become (cb c0 - sb c2, sb c0 + cb c2)
    const float y00 = P.r00 * cb - x02 * sb, y02 = P.r00 * sb + x02 * cb;
    const float y10 = P.r10 * cb - x12 * sb, y12 = P.r10 * sb + x12 * cb;
    const float y20 = P.r20 * cb - x22 * sb, y22 = P.r20 * sb + x22 * cb;
    // * Rz(c): columns 0, 1 become (cc c0 + sc c1, cc c1 - sc c0)
    Frame W;
    W.r00 = y00 * cc + x01 * sc;
    W.r01 = x01 * cc - y00 * sc;
    W.r02 = y02;
    W.r10 = y10 * cc + x11 * sc;
    W.r11 = x11 * cc - y10 * sc;
    W.r12 = y12;
    W.r20 = y20 * cc + x21 * sc;
    W.r21 = x21 * cc - y20 * sc;
    W.r22 = y22;
    W.px = P.px + len * W.r00;
    W.py = P.py + len * W.r10;
    W.pz = P.pz + len * W.r20;
    return W;
}

template <int HW>
__device__ __forceinline__ Frame child_frame_fast_seq(const Frame& P, float a, float b, float c, float len)
{
    float sa, ca, sb, cb, sc, cc;
    sincos_fast<HW>(a, &sa, &ca);
    sincos_fast<HW>(b, &sb, &cb);
    sincos_fast<HW>(c, &sc, &cc);
    return child_frame_fast_seq_sc(P, sa, ca, sb, cb, sc, cc, len);
}

// REFERENCE: the exact sequence of roundings of the reference's
// I*Rx*Ry*Rz*T(len) followed by parent*local 4x4 products
// (src/kernel.cu:52-56, src/matrix_operations.cuh:20-38,123-180) with every
// product by an exact 0 or 1 elided (they do not change a finite value), and
// no FMA contraction.
__device__ __forceinline__ Frame child_frame_reference(const Frame& P, float a, float b, float c, float len)
{
#pragma clang fp contract(off)
    float sa, ca, sb, cb, sc, cc;
    // one fp64 evaluation at a time: interleaving three keeps ~3x the 64-bit
    // temporaries live and spills the particle state
    sincos_reference(a, &sa, &ca);
    __builtin_amdgcn_sched_barrier(0);
    sincos_reference(b, &sb, &cb);
    __builtin_amdgcn_sched_barrier(0);
    sincos_reference(c, &sc, &cc);
    __builtin_amdgcn_sched_barrier(0);
    // A2 = Rx(a) * Ry(b)
    const float a00 = cb, a02 = sb;
    const float a10 = sa * sb, a11 = ca, a12 = (-sa) * cb;
    const float a20 = ca * (-sb), a21 = sa, a22 = ca * cb;
    // A3 = A2 * Rz(c)
    const float l00 = a00 * cc, l01 = a00 * (-sc), l02 = a02;
    const float l10 = a10 * cc + a11 * sc, l11 = a10 * (-sc) + a11 * cc, l12 = a12;
    const float l20 = a20 * cc + a21 * sc, l21 = a20 * (-sc) + a21 * cc, l22 = a22;
    // * T(len, 0, 0): translation column = first column * len
    const float t0 = l00 * len, t1 = l10 * len, t2 = l20 * len;
    Frame W;
    W.r00 = P.r00 * l00 + P.r01 * l10 + P.r02 * l20;
    W.r01 = P.r00 * l01 + P.r01 * l11 + P.r02 * l21;
    W.r02 = P.r00 * l02 + P.r01 * l12 + P.r02 * l22;
    W.r10 = P.r10 * l00 + P.r11 * l10 + P.r12 * l20;
    W.r11 = P.r10 * l01 + P.r11 * l11 + P.r12 * l21;
    W.r12 = P.r10 * l02 + P.r11 * l12 + P.r12 * l22;
    W.r20 = P.r20 * l00 + P.r21 * l10 + P.r22 * l20;
    W.r21 = P.r20 * l01 + P.r21 * l11 + P.r22 * l21;
    W.r22 = P.r20 * l02 + P.r21 * l12 + P.r22 * l22;
    W.px = P.r00 * t0 + P.r01 * t1 + P.r02 * t2 + P.px;
    W.py = P.r10 * t0 + P.r11 * t1 + P.r12 * t2 + P.py;
    W.pz = P.r20 * t0 + P.r21 * t1 + P.r22 * t2 + P.pz;
    return W;
}

// FAST, a node whose parent is the origin, in the origin's own frame: R = Rx(a)
// Ry(b) Rz(c) in closed form (14 operations instead of 36 that would rotate the
// origin's columns) and p = len R e_x.  The kOriginFrame builds move the
// targets into the origin frame at staging, t' = M0^T (t - p0): distances, and
// with them the fitness and the residual, are unchanged by the rigid motion.
__device__ __forceinline__ Frame root_frame_sc(float sa, float ca, float sb, float cb, float sc, float cc, float len)
{
    const float p = sa * sb, q = ca * sb;
    Frame W;
    W.r00 = cb * cc;
    W.r01 = -cb * sc;
    W.r02 = sb;
    W.r10 = p * cc + ca * sc;
    W.r11 = ca * cc - p * sc;
    W.r12 = -sa * cb;
    W.r20 = sa * sc - q * cc;
    W.r21 = q * sc + sa * cc;
    W.r22 = ca * cb;
    W.px = len * W.r00;
    W.py = len * W.r10;
    W.pz = len * W.r20;
    return W;
}

// FAST with every rounding pinned (the collider builds): the same column rotations
// as child_frame_fast_seq_sc and the same closed form as root_frame_sc, with each
// multiply-add written as the fma it is and contraction off, so every kernel that
// evaluates a frame -- the solve's step, its initial fitness, the evaluate kernel --
// computes it bit for bit alike, whatever the compiler would fuse in its context.
// The collider term makes a discrete decision on the frames (GJK), and PSO drives
// answers onto an obstacle's surface, where one ulp decides contact.
__device__ __forceinline__ Frame child_frame_pinned_sc(const Frame& P, float sa, float ca, float sb, float cb,
                                                       float sc, float cc, float len)
{
#pragma clang fp contract(off)
    const float x01 = __builtin_fmaf(P.r02, sa, P.r01 * ca), x02 = __builtin_fmaf(-P.r01, sa, P.r02 * ca);
    const float x11 = __builtin_fmaf(P.r12, sa, P.r11 * ca), x12 = __builtin_fmaf(-P.r11, sa, P.r12 * ca);
    const float x21 = __builtin_fmaf(P.r22, sa, P.r21 * ca), x22 = __builtin_fmaf(-P.r21, sa, P.r22 * ca);
    const float y00 = __builtin_fmaf(-x02, sb, P.r00 * cb), y02 = __builtin_fmaf(x02, cb, P.r00 * sb);
    const float y10 = __builtin_fmaf(-x12, sb, P.r10 * cb), y12 = __builtin_fmaf(x12, cb, P.r10 * sb);
    const float y20 = __builtin_fmaf(-x22, sb, P.r20 * cb), y22 = __builtin_fmaf(x22, cb, P.r20 * sb);
    Frame W;
    W.r00 = __builtin_fmaf(x01, sc, y00 * cc);
    W.r01 = __builtin_fmaf(-y00, sc, x01 * cc);
    W.r02 = y02;
    W.r10 = __builtin_fmaf(x11, sc, y10 * cc);
    W.r11 = __builtin_fmaf(-y10, sc, x11 * cc);
    W.r12 = y12;
    W.r20 = __builtin_fmaf(x21, sc, y20 * cc);
    W.r21 = __builtin_fmaf(-y20, sc, x21 * cc);
    W.r22 = y22;
    W.px = __builtin_fmaf(len, W.r00, P.px);
    W.py = __builtin_fmaf(len, W.r10, P.py);
    W.pz = __builtin_fmaf(len, W.r20, P.pz);
    return W;
}

__device__ __forceinline__ Frame root_frame_pinned_sc(float sa, float ca, float sb, float cb, float sc, float cc,
                                                      float len)
{
#pragma clang fp contract(off)
    const float p = sa * sb, q = ca * sb;
    Frame W;
    W.r00 = cb * cc;
    W.r01 = -(cb * sc);
    W.r02 = sb;
    W.r10 = __builtin_fmaf(ca, sc, p * cc);
    W.r11 = __builtin_fmaf(-p, sc, ca * cc);
    W.r12 = -(sa * cb);
    W.r20 = __builtin_fmaf(-q, cc, sa * sc);
    W.r21 = __builtin_fmaf(sa, cc, q * sc);
    W.r22 = ca * cb;
    W.px = len * W.r00;
    W.py = len * W.r10;
    W.pz = len * W.r20;
    return W;
}

// SEQ: FAST mode may compose the rotation column-wise (interior nodes, or any
// node whose full frame is consumed).  HW: FAST sin/cos on the transcendental unit.
template <int MODE, bool SEQ = false, int HW = kTrigPoly>
__device__ __forceinline__ Frame child_frame(const Frame& P, float a, float b, float c, float len)
{
    if constexpr (MODE == IKPSO_ARITH_REFERENCE)
        return child_frame_reference(P, a, b, c, len);
    else if constexpr (SEQ)
        return child_frame_fast_seq<HW>(P, a, b, c, len);
    else
        return child_frame_fast<HW>(P, a, b, c, len);
}

// ---------------------------------------------------------------- fitness
// calculateDistance (src/kernel.cu:64-151) for one particle:
//   f = sum_eff w_e |p_e - t_e|^2 + (dw/J) sum_k |(p_k,1) - posref_k|^2
//       + (aw/J) sum_k |rest_k - x_k|^2   [+ soft joint-limit penalty, extension]
// Accumulation order follows the reference (node order; (x^2+y^2)+z^2).
// `tgt` holds the effector targets per node (3 floats at 3*(k-1)); for the
// generic topology non-effector nodes carry weight 0 and target 0, and adding
// the resulting +0 leaves a finite sum unchanged bit for bit.
// TERMS: which optional terms are compiled in -- kTermPosRef (distanceWeight
// != 0: the positions[] term), kTermPenalty (soft joint limits), or
// kTermRuntime (generic kernels: both decided by runtime flags);
// kTermUniformBounds: every angle has the same clamp bounds (the reference
// scene: [0, 2pi] on every axis), read once from the kernarg into SGPRs
// instead of per dimension from LDS.
// kTermColliders: the collider (GJK) block of calculateDistance
// (src/kernel.cu:104-136), compiled in only when the scene has colliders.
// kTermMask: the chain has a joint-axis mask (ChainConsts::free_mask): locked
// angles take no draws and no update (uniform branches per dimension, which
// cost the register allocator enough that unmasked chains get builds without).
// kTermRev: the kernel keeps its angles in revolutions (x / 2pi): positions,
// velocities, local and global bests, rest angles, clamp and soft limits, so the
// transcendental unit's v_sin / v_cos take them as they are (kTrigHwRev: one
// multiply fewer per angle); the angle and penalty weights carry the (2 pi)^2,
// and the answers are scaled back by 2 pi on the way out.  Only the resident
// and cooperative FAST builds with the hardware sin/cos (the streaming kernels
// keep the reference's radian layout in HBM).
constexpr int kTermPosRef = 1, kTermPenalty = 2, kTermRuntime = 4, kTermUniformBounds = 8, kTermColliders = 16,
              kTermMask = 32, kTermRev = 64, kTermUnitBounds = 128, kTermSymPenalty = 256;
// kTermUnitBounds (with kTermRev and kTermUniformBounds): the clamp bounds are
// exactly [0, 1] revolutions -- the reference scene's [0, 2pi] -- so the clamp
// is the VALU's free output clamp on the position update instead of a v_med3
// (half rate on gfx950).
// kTermSymPenalty (with kTermRev and kTermPenalty): the soft limits are
// symmetric, soft_lo = -soft_hi, and every clamped angle lies within one
// revolution of them, so the penalty's overshoot max(|x| - h, 0) is the VALU's
// free output clamp of |x| - h (<= 1) instead of two subtractions and a v_max3
// (half rate): BASELINE config 5's +-pi/2 soft limits inside +-pi.

// Parity-attribution builds of FAST arithmetic (tools/tier_b_attribution.py; built into
// variants/, never shipped): each switch removes one FAST ingredient --
//   IKPSO_FAST_REV=0            angles in radians (no kTermRev, so no revolution-unit clamp,
//                               symmetric-penalty clamp or origin-frame FK either);
//   IKPSO_FAST_HW_TRIG=0        the 1-ulp polynomial instead of v_sin / v_cos;
//   IKPSO_FAST_TIP_BACKWARD=0   the tip-effector serial chains evaluate their FK forward.
#ifndef IKPSO_FAST_REV
#define IKPSO_FAST_REV 1
#endif
#ifndef IKPSO_FAST_HW_TRIG
#define IKPSO_FAST_HW_TRIG 1
#endif
#ifndef IKPSO_FAST_TIP_BACKWARD
#define IKPSO_FAST_TIP_BACKWARD 1
#endif
// the revolution-unit terms of the specialised FAST builds (0 in an IKPSO_FAST_REV=0 build)
constexpr int kFastRev = IKPSO_FAST_REV ? kTermRev : 0;
constexpr int kFastUnitBounds = IKPSO_FAST_REV ? kTermUnitBounds : 0;
constexpr int kFastSymPenalty = IKPSO_FAST_REV ? kTermSymPenalty : 0;

// Generator type of a swarm kernel: the add-for-shift issue form everywhere but
// in the collider kernels, whose register allocation the opaque add perturbs
// (spills); the draws are bit-identical either way.
template <int TERMS>
using RngFor = XorwowT<!(TERMS & kTermColliders)>;

// FAST sin/cos on the transcendental unit (sincos_fast<true>) for a kernel of
// this topology and term set (D <= 60); of the collider builds the unmasked ones
// of the compiled topologies (IKPSO_COLLIDE_HW_TRIG; the generic trees' collider
// builds trip a hipcc 7.2 backend error with it -- "Illegal instruction detected:
// Operand has incorrect register class", a flat-to-private check -- and keep the
// polynomial).
// The unmasked collider builds on the transcendental unit too (round 6; round 5
// kept them on the polynomial because the solve and evaluate kernels then disagreed
// on contact decisions: the compiler's FMA contraction of the same frame code
// differed between the kernels -- FitnessAcc::kPin now pins every rounding).  The
// masked collider builds keep the polynomial, and carry the chains whose angles
// reach beyond the unit's range (ChainHost::poly_trig).  0: round 5's builds.
#ifndef IKPSO_COLLIDE_HW_TRIG
#define IKPSO_COLLIDE_HW_TRIG 1
#endif
// FAST collider builds test the near nodes by separating axes (node_collides_obb) instead
// of the reference's GJK: the same routing as the transcendental unit's (unmasked, compiled
// topologies); the host sends chains whose colliders are not rotations to the masked builds
// (ChainHost::coll_obb).  0: GJK in every build.
#ifndef IKPSO_FAST_SAT
#define IKPSO_FAST_SAT 1
#endif
#ifndef IKPSO_CAND_COMPACT
#define IKPSO_CAND_COMPACT 1
#endif
template <class Topo, int MODE, int TERMS>
constexpr bool kFastSat = IKPSO_FAST_SAT && MODE == IKPSO_ARITH_FAST && (TERMS & kTermColliders) &&
                          !(TERMS & kTermMask) && !Topo::kGeneric;
template <class Topo, int MODE, int TERMS>
constexpr bool kHwTrigOk = IKPSO_FAST_HW_TRIG && MODE == IKPSO_ARITH_FAST && Topo::D <= 60 &&
                           (!(TERMS & kTermColliders) ||
                            (IKPSO_COLLIDE_HW_TRIG && !(TERMS & kTermMask) && !Topo::kGeneric));
// The sin/cos flavour of a kernel build (sincos_fast): polynomial, hardware on
// radians, or hardware on revolutions (kTermRev).
template <class Topo, int MODE, int TERMS>
constexpr int kHwTrig = !kHwTrigOk<Topo, MODE, TERMS> ? ((TERMS & kTermRev) ? kTrigPolyRev : kTrigPoly)
                       : (TERMS & kTermRev) ? kTrigHwRev : kTrigHw;
template <class Topo, int MODE, int TERMS>
constexpr bool kRev = (TERMS & kTermRev) != 0;
// Link k's length for a build whose sin/cos flavour is HW: the transcendental
// unit's builds read the lengths compensated for its amplitude bias
// (ChainConsts::len_hw, kHwTrigAmplitudeBias), every other build the chain's own.
template <int HW, class CC>
__device__ __forceinline__ float link_len(const CC& cc, int k)
{
    return (HW == kTrigHw || HW == kTrigHwRev) ? cc.len_hw[k] : cc.len[k];
}
// angle / penalty weights of a build (kTermRev: the (2 pi)^2 of the revolution units)
template <int TERMS, class CC>
__device__ __forceinline__ float angle_weight(const CC& cc) { return (TERMS & kTermRev) ? cc.aw_rev : cc.aw_j; }
template <int TERMS, class CC>
__device__ __forceinline__ float limit_weight(const CC& cc) { return (TERMS & kTermRev) ? cc.lim_rev : cc.lim_w; }
constexpr float kInv2Pi = 0.159154943091895336f, k2Pi = 6.28318530717958648f;
// the uniform clamp bounds (kTermUniformBounds) in the build's angle units
// Euler topologies of the kTermRev builds evaluate their FK in the origin's
// frame (root_frame_sc): the swarm kernels stage the targets moved into it.
template <class Topo, int TERMS>
constexpr bool kOriginFrame = (TERMS & kTermRev) && !Topo::kDH && !Topo::kGeneric;
template <int TERMS, class CC>
__device__ __forceinline__ float uniform_lo(const CC& cc)
{
    if constexpr (TERMS & kTermUnitBounds) return 0.0f;
    return (TERMS & kTermRev) ? cc.rlo : cc.lo[0];
}
template <int TERMS, class CC>
__device__ __forceinline__ float uniform_hi(const CC& cc)
{
    if constexpr (TERMS & kTermUnitBounds) return 1.0f;
    return (TERMS & kTermRev) ? cc.rhi : cc.hi[0];
}

// Which kernel builds honour ChainConsts::free_mask (the host routes masked
// chains to them; the folded chain has no locked angles).
template <class Topo, int TERMS>
constexpr bool kMasked = (TERMS & kTermMask) && !Topo::kDH;


#if IKPSO_COLLIDE_STATS
#define IKPSO_CC_STATS , cc.coll_stats
#else
#define IKPSO_CC_STATS
#endif
template <class Topo, int MODE, int TERMS>
struct FitnessAcc {
    static constexpr int J = Topo::J;
    Frame F[J + 1];
    const float* soft;  // soft limits [lo 3J | hi 3J]: the swarm kernels' LDS copy, else aux in HBM
    float rot_diff, pos_diff, distance, pen;
    bool posref, penalty;
    // kTermColliders: the nodes whose boxes may touch a collider (bit k-1), and their
    // frames -- rotation, position, parent position, link length -- for finish(), in
    // the caller's CandBuf (a separate private array: indexed at run time by finish,
    // it lives in scratch, and only the near nodes' frames are written to it).
    // Generic trees test a near node at once (hit): their deferred build hits a
    // hipcc 7.2 backend error (a flat-to-private check on the buffer's address).
    static constexpr bool kDefer = (TERMS & kTermColliders) && !Topo::kGeneric;
    // FAST collider builds pin every rounding of the frames and of the fitness sums
    // (child_frame_pinned_sc): the contact decisions of one arithmetic must not
    // depend on the kernel that makes them
    static constexpr bool kPin = (TERMS & kTermColliders) && MODE == IKPSO_ARITH_FAST;
    // The separating-axis builds store a near node's frame as two axes and its position
    // (9 floats instead of 16: the scratch traffic of the stored frames); the third axis
    // is their cross product and the parent's position p - len R e_x, both recomputed
    // in finish_for_update by every kernel alike (IKPSO_CAND_COMPACT).
    static constexpr bool kCompactCand = IKPSO_CAND_COMPACT && kFastSat<Topo, MODE, TERMS> && kDefer;
    uint32_t near_mask;
    float* cand;
    bool hit;
    const float* nearc = nullptr;  // the swarm kernels' SwarmShared::near4 (near_collider_lds), else null

    // soft_: the soft limits -- pass the swarm kernel's LDS copy (SwarmShared::soft)
    // where there is one: a pointer that may be LDS or global is a flat pointer
    __device__ __forceinline__ FitnessAcc(const ChainConsts<J>& cc, const float*, const float* soft_, float* cand_)
        : soft(soft_), rot_diff(0.0f), pos_diff(0.0f), distance(0.0f), pen(0.0f),
          posref((TERMS & kTermPosRef) || ((TERMS & kTermRuntime) && cc.use_posref)),
          penalty((TERMS & kTermPenalty) || ((TERMS & kTermRuntime) && cc.use_penalty)), near_mask(0u),
          cand(cand_), hit(false)
    {
        F[0] = origin_frame(cc.m0);
    }

    // Node k (1..J) with its three Euler angles, its three rest angles and (for
    // effectors) its target; nodes must come in index order.
    // column-wise composition unless only the leaf's position is consumed
    __device__ __forceinline__ static constexpr bool seq(int k)
    {
        return !Topo::kGeneric && (!Topo::leaf(k) || (TERMS & kTermColliders));
    }

    __device__ __forceinline__ void node(const ChainConsts<J>& cc, int k, float a, float b, float c,
                                         const float* rest3, const float* tgt3, float* node_pos)
    {
        const int pk = Topo::kGeneric ? cc.parent[k] : Topo::parent(k);
        constexpr int HW = kHwTrig<Topo, MODE, TERMS>;
        if constexpr (kPin) {  // FAST collider builds: every rounding pinned (child_frame_pinned_sc)
            float sa, ca, sb, cb, sc, cc_;
            sincos_fast<HW>(a, &sa, &ca);
            sincos_fast<HW>(b, &sb, &cb);
            sincos_fast<HW>(c, &sc, &cc_);
            if (kOriginFrame<Topo, TERMS> && pk == 0)
                F[k] = root_frame_pinned_sc(sa, ca, sb, cb, sc, cc_, link_len<HW>(cc, k));
            else
                F[k] = child_frame_pinned_sc(F[pk], sa, ca, sb, cb, sc, cc_, link_len<HW>(cc, k));
        } else if (kOriginFrame<Topo, TERMS> && pk == 0) {
            float sa, ca, sb, cb, sc, cc_;
            sincos_fast<HW>(a, &sa, &ca);
            sincos_fast<HW>(b, &sb, &cb);
            sincos_fast<HW>(c, &sc, &cc_);
            F[k] = root_frame_sc(sa, ca, sb, cb, sc, cc_, link_len<HW>(cc, k));
        } else if (seq(k)) {
            F[k] = child_frame<MODE, true, HW>(F[pk], a, b, c, link_len<HW>(cc, k));
        } else {
            F[k] = child_frame<MODE, false, HW>(F[pk], a, b, c, link_len<HW>(cc, k));
        }
        terms(cc, k, a, b, c, rest3, tgt3, node_pos);
    }

    // FAST, with the node's sines and cosines computed ahead (node_trig).
    __device__ __forceinline__ void node_trig(const ChainConsts<J>& cc, int k, const float* ang, const NodeTrig<3>& t,
                                              const float* rest3, const float* tgt3, float* node_pos)
    {
        static_assert(MODE == IKPSO_ARITH_FAST, "precomputed sin/cos: FAST arithmetic");
        const int pk = Topo::kGeneric ? cc.parent[k] : Topo::parent(k);
        constexpr int HW = kHwTrig<Topo, MODE, TERMS>;
        const float len = link_len<HW>(cc, k);
        if (kOriginFrame<Topo, TERMS> && pk == 0)
            F[k] = root_frame_sc(t.s[0], t.c[0], t.s[1], t.c[1], t.s[2], t.c[2], len);
        else if (seq(k))
            F[k] = child_frame_fast_seq_sc(F[pk], t.s[0], t.c[0], t.s[1], t.c[1], t.s[2], t.c[2], len);
        else
            F[k] = child_frame_fast_sc(F[pk], t.s[0], t.c[0], t.s[1], t.c[1], t.s[2], t.c[2], len);
        terms(cc, k, ang[0], ang[1], ang[2], rest3, tgt3, node_pos);
    }

    // The fitness terms of node k once its frame F[k] is known.
    __device__ __forceinline__ void terms(const ChainConsts<J>& cc, int k, float a, float b, float c,
                                          const float* rest3, const float* tgt3, float* node_pos)
    {
#pragma clang fp contract(off)
        const int pk = Topo::kGeneric ? cc.parent[k] : Topo::parent(k);
        const float dx = rest3[0] - a, dy = rest3[1] - b, dz = rest3[2] - c;
        if constexpr (MODE == IKPSO_ARITH_REFERENCE) {
            rot_diff = rot_diff + ((dx * dx + dy * dy) + dz * dz);
        } else if constexpr (kPin) {
            rot_diff = rot_diff + __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
        } else {
#pragma clang fp contract(fast)
            rot_diff = rot_diff + ((dx * dx + dy * dy) + dz * dz);
        }
        if (posref) {  // distance_weight != 0
            const float* pr = cc.aux + 4 * (k - 1);  // positions[(k-1)*4 ..] (src/kernel.cu:94-98)
            const float ex = F[k].px - pr[0];
            const float ey = F[k].py - pr[1];
            const float ez = F[k].pz - pr[2];
            const float ew = 1.0f - pr[3];
            pos_diff += ((ex * ex + ey * ey) + ez * ez) + ew * ew;
        }
        if (Topo::effector(k)) {
            const float ex = F[k].px - tgt3[0];
            const float ey = F[k].py - tgt3[1];
            const float ez = F[k].pz - tgt3[2];
            if constexpr (MODE == IKPSO_ARITH_REFERENCE) {
                distance = distance + ((ex * ex + ey * ey) + ez * ez) * cc.eff_w[k];
            } else if constexpr (kPin) {
                distance = __builtin_fmaf(__builtin_fmaf(ez, ez, __builtin_fmaf(ey, ey, ex * ex)), cc.eff_w[k], distance);
            } else {
#pragma clang fp contract(fast)
                distance = distance + ((ex * ex + ey * ey) + ez * ez) * cc.eff_w[k];
            }
        }
        if (penalty) {  // soft joint-limit penalty (extension, BASELINE config 5), d order
            const float ang[3] = {a, b, c};
#pragma unroll
            for (int ax = 0; ax < 3; ++ax) {
                const int d = 3 * (k - 1) + ax;
                const float slo = soft[d], shi = soft[3 * J + d];
                const float over = fmaxf(fmaxf(ang[ax] - shi, slo - ang[ax]), 0.0f);
                pen = pen + over * over;
            }
        }
        if constexpr (TERMS & kTermColliders) {
            // The inline sphere test on the node's and its parent's positions; a node
            // that passes it keeps its frame for the quaternion and GJK part, which
            // finish() runs after the last node (see there).  No colliders: a chain
            // routed here for its polynomial sin/cos (ChainHost::poly_trig).
            if (!kDefer) {
                if (!hit && cc.num_coll > 0 &&
                    near_collider(F[k].px, F[k].py, F[k].pz, F[pk].px, F[pk].py, F[pk].pz,
                                  cc.coll_lim + (k - 1) * cc.num_coll, cc.coll, cc.num_coll IKPSO_CC_STATS))
                    hit = node_collides(F[k].r00, F[k].r01, F[k].r02, F[k].r10, F[k].r11, F[k].r12, F[k].r20,
                                        F[k].r21, F[k].r22, F[k].px, F[k].py, F[k].pz, F[pk].px, F[pk].py, F[pk].pz,
                                        cc.len[k], cc.coll, cc.num_coll IKPSO_CC_STATS);
            } else if (cc.num_coll > 0 &&
                       (nearc ? near_collider_lds(F[k].px, F[k].py, F[k].pz, F[pk].px, F[pk].py, F[pk].pz,
                                                  nearc + 4 * kNearUnroll * (k - 1),
                                                  cc.coll_lim + (k - 1) * cc.num_coll, cc.coll, cc.num_coll)
                              : near_collider(F[k].px, F[k].py, F[k].pz, F[pk].px, F[pk].py, F[pk].pz,
                                              cc.coll_lim + (k - 1) * cc.num_coll, cc.coll,
                                              cc.num_coll IKPSO_CC_STATS))) {
                near_mask |= 1u << (k - 1);
                float* c = cand + 16 * (k - 1);
                if constexpr (kCompactCand) {  // two axes and the position (finish_for_update rebuilds the rest)
                    c[0] = F[k].r00, c[1] = F[k].r10, c[2] = F[k].r20;
                    c[3] = F[k].r01, c[4] = F[k].r11, c[5] = F[k].r21;
                    c[6] = F[k].px, c[7] = F[k].py, c[8] = F[k].pz;
                } else {
                    c[0] = F[k].r00, c[1] = F[k].r01, c[2] = F[k].r02;
                    c[3] = F[k].r10, c[4] = F[k].r11, c[5] = F[k].r12;
                    c[6] = F[k].r20, c[7] = F[k].r21, c[8] = F[k].r22;
                    c[9] = F[k].px, c[10] = F[k].py, c[11] = F[k].pz;
                    c[12] = F[pk].px, c[13] = F[pk].py, c[14] = F[pk].pz;
                    c[15] = cc.len[k];
                }
            }
        }
        if (node_pos) {
            node_pos[3 * (k - 1) + 0] = F[k].px;
            node_pos[3 * (k - 1) + 1] = F[k].py;
            node_pos[3 * (k - 1) + 2] = F[k].pz;
        }
    }

    // The same with the node's angles, rest angles and target by pointer.
    __device__ __forceinline__ void node(const ChainConsts<J>& cc, int k, const float* ang, const float* rest3,
                                         const float* tgt3, float* node_pos)
    {
        node(cc, k, ang[0], ang[1], ang[2], rest3, tgt3, node_pos);
    }

    // Any node/link box hit -> FLT_MAX (the reference returns at its first hit; a
    // hit is a hit in any node order).  The quaternion and GJK part (node_collides,
    // out of line) runs here, once per near node, after the FK pass: a call inside
    // the pass made every value live across it a spill candidate, and the pass
    // paid for the spills whether or not a lane came near (round 5: the boxes out
    // of reach, 214 ms with the call in the pass vs 79 ms without it).
    // finish(cc): the fitness itself (every lane tested).  finish_for_update(cc,
    // pbest): a value valid ONLY for the strict `f < pbest` local-best update
    // (updateLocalBests, src/kernel.cu:202-221) -- a lane whose collision-free value
    // is already >= a finite pbest cannot improve whether or not it collides
    // (FLT_MAX is not < pbest either), so it skips the test and returns that value:
    // the update, and so every later state, is the same bit for bit, but the value
    // itself may be the collision-free one.  A call site that keeps f as a fitness
    // (an initial local best, a reported or evaluated fitness) must use finish(cc).
    __device__ __forceinline__ float finish(const ChainConsts<J>& cc) const
    {
        return finish_for_update(cc, __builtin_nanf(""));  // NaN: no lane skips
    }

    __device__ __forceinline__ float finish_for_update(const ChainConsts<J>& cc, float pbest) const
    {
#pragma clang fp contract(off)
        const float aw = angle_weight<TERMS>(cc);
        float f = posref ? (distance + cc.dw_j * pos_diff) + aw * rot_diff : distance + aw * rot_diff;
        if (penalty) f = f + limit_weight<TERMS>(cc) * pen;
        if constexpr (TERMS & kTermColliders) {
            if (hit) f = FLT_MAX;  // (generic trees)
            uint32_t m = (f >= pbest && pbest <= FLT_MAX) ? 0u : near_mask;
            while (m != 0u) {
                const int slot = __builtin_ctz(m);  // node slot + 1 = k
                const float* c = cand + 16 * slot;
                m &= m - 1u;
                if constexpr (kCompactCand) {
                    const int k = slot + 1;
                    constexpr int HW = kHwTrig<Topo, MODE, TERMS>;
                    const float a0 = c[0], a1 = c[1], a2 = c[2], b0 = c[3], b1 = c[4], b2 = c[5];
                    const float e0 = a1 * b2 - a2 * b1, e1 = a2 * b0 - a0 * b2, e2 = a0 * b1 - a1 * b0;
                    const float l = link_len<HW>(cc, k);
                    const float qx = c[6] - l * a0, qy = c[7] - l * a1, qz = c[8] - l * a2;
                    if (node_collides_obb(a0, b0, e0, a1, b1, e1, a2, b2, e2, c[6], c[7], c[8], qx, qy, qz, cc.len[k],
                                          cc.coll, cc.coll_box, cc.num_coll)) {
                        f = FLT_MAX;
                        break;
                    }
                } else if constexpr (kFastSat<Topo, MODE, TERMS>) {
                    if (node_collides_obb(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8], c[9], c[10], c[11],
                                          c[12], c[13], c[14], c[15], cc.coll, cc.coll_box, cc.num_coll)) {
                        f = FLT_MAX;
                        break;
                    }
                } else if (node_collides(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8], c[9], c[10], c[11],
                                         c[12], c[13], c[14], c[15], cc.coll, cc.num_coll IKPSO_CC_STATS)) {
                    f = FLT_MAX;
                    break;
                }
            }
        }
        return f;
    }
};

// FK + fitness of the folded serial chain (TopoDH; FAST arithmetic): the tip
// effector term, the angle term over the free angles and the soft-limit
// penalty -- calculateDistance (src/kernel.cu:64-151) of the chain with its
// locked angles at rest (the locked angles add exact zeros to the angle term).
// No distance or collider term (the host routes those chains to the Euler
// kernels).  `dhc` = the folded chain's constants (12 floats per joint + q0;
// ChainConsts::dh_off): the swarm kernels' LDS copy, passed unconditionally so
// the loads stay ds_read (a pointer that may be LDS or global is a flat pointer,
// and flat loads of LDS data cost vector-memory latency).
template <class Topo, int MODE, int TERMS>
struct FitnessAccDH {
    static constexpr int J = Topo::J;
    static constexpr int HW = kHwTrig<Topo, MODE, TERMS>;
    static_assert(MODE == IKPSO_ARITH_FAST, "the folded chain is FAST arithmetic only");
    const float* dhc;
    const float* soft;                                  // soft limits [lo 3J | hi 3J] (see FitnessAcc)
    float w00, w01, w02, w10, w11, w12, w20, w21, w22;  // current joint frame W_j
    float qx, qy, qz;                                   // position q_j
    float px, py, pz;                                   // tip (after joint J)
    float rot_diff, distance, pen;
    bool penalty;

    __device__ __forceinline__ FitnessAccDH(const ChainConsts<J>& cc, const float* dh, const float* soft_, float*)
        : dhc(dh), soft(soft_), rot_diff(0.0f), distance(0.0f), pen(0.0f),
          penalty((TERMS & kTermPenalty) || ((TERMS & kTermRuntime) && cc.use_penalty))
    {
        qx = dhc[12 * J + 0];
        qy = dhc[12 * J + 1];
        qz = dhc[12 * J + 2];
    }

    // Joint k (1..J) at angle t: W = W * C_k * Rz(t), then q += W s_k.
    __device__ __forceinline__ void advance(int k, float t)
    {
        float st, ct;
        sincos_fast<HW>(t, &st, &ct);
        advance_sc(k, st, ct);
    }

    __device__ __forceinline__ void advance_sc(int k, float st, float ct)
    {
        const float* C = dhc + 12 * (k - 1);
        float m00, m01, m02, m10, m11, m12, m20, m21, m22;
        if (k == 1) {
            m00 = C[0]; m01 = C[1]; m02 = C[2];
            m10 = C[3]; m11 = C[4]; m12 = C[5];
            m20 = C[6]; m21 = C[7]; m22 = C[8];
        } else {
            const float c00 = C[0], c01 = C[1], c02 = C[2], c10 = C[3], c11 = C[4], c12 = C[5], c20 = C[6],
                        c21 = C[7], c22 = C[8];
            m00 = w00 * c00 + w01 * c10 + w02 * c20;
            m01 = w00 * c01 + w01 * c11 + w02 * c21;
            m02 = w00 * c02 + w01 * c12 + w02 * c22;
            m10 = w10 * c00 + w11 * c10 + w12 * c20;
            m11 = w10 * c01 + w11 * c11 + w12 * c21;
            m12 = w10 * c02 + w11 * c12 + w12 * c22;
            m20 = w20 * c00 + w21 * c10 + w22 * c20;
            m21 = w20 * c01 + w21 * c11 + w22 * c21;
            m22 = w20 * c02 + w21 * c12 + w22 * c22;
        }
        const float s0 = C[9], s1 = C[10], s2 = C[11];
        if (k == J) {
            // the tip only needs W s = M (Rz(t) s)
            const float v0 = ct * s0 - st * s1, v1 = st * s0 + ct * s1;
            px = qx + m00 * v0 + m01 * v1 + m02 * s2;
            py = qy + m10 * v0 + m11 * v1 + m12 * s2;
            pz = qz + m20 * v0 + m21 * v1 + m22 * s2;
        } else {
            // * Rz(t): columns 0, 1 become (ct c0 + st c1, ct c1 - st c0)
            w00 = ct * m00 + st * m01; w01 = ct * m01 - st * m00; w02 = m02;
            w10 = ct * m10 + st * m11; w11 = ct * m11 - st * m10; w12 = m12;
            w20 = ct * m20 + st * m21; w21 = ct * m21 - st * m20; w22 = m22;
            qx = qx + w00 * s0 + w01 * s1 + w02 * s2;
            qy = qy + w10 * s0 + w11 * s1 + w12 * s2;
            qz = qz + w20 * s0 + w21 * s1 + w22 * s2;
        }
    }

    // Joint k with its one angle, rest angle and (tip) target.
    __device__ __forceinline__ void node(const ChainConsts<J>& cc, int k, const float* ang, const float* rest,
                                         const float* tgt3, float* node_pos)
    {
        advance(k, ang[0]);
        terms(cc, k, ang[0], rest, tgt3, node_pos);
    }

    __device__ __forceinline__ void node_trig(const ChainConsts<J>& cc, int k, const float* ang, const NodeTrig<1>& t,
                                              const float* rest, const float* tgt3, float* node_pos)
    {
        advance_sc(k, t.s[0], t.c[0]);
        terms(cc, k, ang[0], rest, tgt3, node_pos);
    }

    __device__ __forceinline__ void terms(const ChainConsts<J>& cc, int k, float t, const float* rest,
                                          const float* tgt3, float* node_pos)
    {
        const float dt = rest[0] - t;
        rot_diff = rot_diff + dt * dt;
        if (penalty) {
            const int d = k - 1;
            const float slo = soft[d], shi = soft[3 * J + d];
            const float over = fmaxf(fmaxf(t - shi, slo - t), 0.0f);
            pen = pen + over * over;
        }
        if (k == J) {
            const float ex = px - tgt3[0], ey = py - tgt3[1], ez = pz - tgt3[2];
            distance = ((ex * ex + ey * ey) + ez * ez) * cc.eff_w[J];
            if (node_pos) {  // [3J]: the tip's slot
                node_pos[3 * (J - 1) + 0] = px;
                node_pos[3 * (J - 1) + 1] = py;
                node_pos[3 * (J - 1) + 2] = pz;
            }
        }
    }

    __device__ __forceinline__ float finish(const ChainConsts<J>& cc) const
    {
        float f = distance + angle_weight<TERMS>(cc) * rot_diff;
        if (penalty) f = f + limit_weight<TERMS>(cc) * pen;
        return f;
    }
    // (no collider term: the value is the fitness itself; FitnessAcc::finish_for_update)
    __device__ __forceinline__ float finish_for_update(const ChainConsts<J>& cc, float) const { return finish(cc); }
};

template <class Topo, int MODE, int TERMS>
using FitnessFor =
    std::conditional_t<Topo::kDH, FitnessAccDH<Topo, MODE, TERMS>, FitnessAcc<Topo, MODE, TERMS>>;
// The near nodes' frames of a FitnessAcc with the collider term (FitnessAcc::cand).
template <class Topo, int TERMS>
struct CandBuf {
    float v[(TERMS & kTermColliders) && !Topo::kDH && !Topo::kGeneric ? 16 * Topo::J : 1];
};

// FAST serial chains whose only position term is the tip (TopoSerialTip; no
// distance term, colliders or mask, terms known at compile time): the tip is
// evaluated from the tip back, in the chain's Horner form
//   p_J = p_0 + R_0 (R_1 (l_1 e_x + R_2 (l_2 e_x + ... R_J (l_J e_x))))
// with R_k = Rx(a) Ry(b) Rz(c): per node three plane rotations of ONE vector
// (12 multiply-adds + 1 add) instead of composing the node's world frame (36
// multiply-adds for the three column rotations + 3 for the position) -- only
// the tip's position is consumed, so no node's frame is needed.  The angle and
// penalty terms accumulate in node order exactly as FitnessAcc::terms does.
template <class Topo>
struct IsSerialTip : std::false_type {};
template <int J>
struct IsSerialTip<TopoSerialTip<J>> : std::true_type {};
template <class Topo, int MODE, int TERMS>
constexpr bool kTipBackward = MODE == IKPSO_ARITH_FAST &&
                              ((IsSerialTip<Topo>::value && IKPSO_FAST_TIP_BACKWARD) || Topo::kDH) &&
                              !(TERMS & (kTermPosRef | kTermRuntime | kTermColliders | kTermMask));

template <class Topo, int MODE, int TERMS>
struct TipBackAcc {
    static constexpr int J = Topo::J;
    static constexpr int HW = kHwTrig<Topo, MODE, TERMS>;
    const float* soft;
    float rot_diff, pen, ux, uy, uz;

    __device__ __forceinline__ TipBackAcc(const float*, const float* soft_) : soft(soft_), rot_diff(0.0f), pen(0.0f) {}

    // node k's angle terms (node order, as FitnessAcc::terms)
    __device__ __forceinline__ void angles(int k, const float* ang, const float* rest3)
    {
        const float dx = rest3[0] - ang[0], dy = rest3[1] - ang[1], dz = rest3[2] - ang[2];
        rot_diff = rot_diff + ((dx * dx + dy * dy) + dz * dz);
        if constexpr (TERMS & kTermPenalty) {
#pragma unroll
            for (int ax = 0; ax < 3; ++ax) {
                const int d = 3 * (k - 1) + ax;
                float over;
                if constexpr (TERMS & kTermSymPenalty)  // |x| - h clamped to [0, 1]: one v_sub with clamp
                    over = __builtin_amdgcn_fmed3f(fabsf(ang[ax]) - soft[3 * J + d], 0.0f, 1.0f);
                else
                    over = fmaxf(fmaxf(ang[ax] - soft[3 * J + d], soft[d] - ang[ax]), 0.0f);
                pen = pen + over * over;
            }
        }
    }

    // u <- R_k (l_k e_x + u); nodes from J down to 1 (node J starts from u = 0)
    __device__ __forceinline__ void back(const ChainConsts<J>& cc, int k, const NodeTrig<3>& t)
    {
        const float sa = t.s[0], ca = t.c[0], sb = t.s[1], cb = t.c[1], sc = t.s[2], cc_ = t.c[2];
        const float l = link_len<HW>(cc, k);
        float w0, w1, w2;
        if (k == J) {  // Rz (l, 0, 0)
            w0 = cc_ * l;
            w1 = sc * l;
            w2 = 0.0f;
        } else {
            const float a0 = ux + l;
            w0 = cc_ * a0 - sc * uy;
            w1 = sc * a0 + cc_ * uy;
            w2 = uz;
        }
        // Ry: (cb w0 + sb w2, w1, cb w2 - sb w0)
        const float y0 = k == J ? cb * w0 : cb * w0 + sb * w2;
        const float y2 = k == J ? -(sb * w0) : cb * w2 - sb * w0;
        // Rx: (y0, ca w1 - sa y2, sa w1 + ca y2)
        ux = y0;
        uy = ca * w1 - sa * y2;
        uz = sa * w1 + ca * y2;
    }

    // fitness once back() has run for node 1: the tip term + the angle terms
    __device__ __forceinline__ float finish(const ChainConsts<J>& cc, const float* tgt3) const
    {
        float px = ux, py = uy, pz = uz;  // kOriginFrame: the target is in the origin frame
        if constexpr (!kOriginFrame<Topo, TERMS>) {
            const float* m = cc.m0;  // origin frame, row-major 3x4
            px = m[3] + (m[0] * ux + m[1] * uy + m[2] * uz);
            py = m[7] + (m[4] * ux + m[5] * uy + m[6] * uz);
            pz = m[11] + (m[8] * ux + m[9] * uy + m[10] * uz);
        }
        const float ex = px - tgt3[0], ey = py - tgt3[1], ez = pz - tgt3[2];
        const float distance = ((ex * ex + ey * ey) + ez * ez) * cc.eff_w[J];
        float f = distance + angle_weight<TERMS>(cc) * rot_diff;
        if constexpr (TERMS & kTermPenalty) f = f + limit_weight<TERMS>(cc) * pen;
        return f;
    }
};

// The folded chain (TopoDH) from the tip back: tip = q_0 + C_1 Rz(t_1) (s_1 +
// C_2 Rz(t_2) (s_2 + ... + C_J Rz(t_J) s_J)) -- per joint 3 adds, one plane
// rotation (4) and C_j times a vector (9) instead of W_{j-1} C_j (27), the
// column rotation (12) and the position (9) of FitnessAccDH.
template <class Topo, int MODE, int TERMS>
struct TipBackAccDH {
    static constexpr int J = Topo::J;
    static constexpr int HW = kHwTrig<Topo, MODE, TERMS>;
    const float* dhc;
    const float* soft;
    float rot_diff, pen, ux, uy, uz;

    __device__ __forceinline__ TipBackAccDH(const float* dh, const float* soft_)
        : dhc(dh), soft(soft_), rot_diff(0.0f), pen(0.0f)
    {
    }

    __device__ __forceinline__ void angles(int k, const float* ang, const float* rest)
    {
        const float dt = rest[0] - ang[0];
        rot_diff = rot_diff + dt * dt;
        if constexpr (TERMS & kTermPenalty) {
            const int d = k - 1;
            const float slo = soft[d], shi = soft[3 * J + d];
            const float over = fmaxf(fmaxf(ang[0] - shi, slo - ang[0]), 0.0f);
            pen = pen + over * over;
        }
    }

    // u <- C_k Rz(t_k) (s_k + u); joints from J down to 1 (joint J: u = 0)
    __device__ __forceinline__ void back(const ChainConsts<J>&, int k, const NodeTrig<1>& t)
    {
        const float* C = dhc + 12 * (k - 1);
        const float st = t.s[0], ct = t.c[0];
        float w0 = C[9], w1 = C[10], w2 = C[11];
        if (k < J) {
            w0 = w0 + ux;
            w1 = w1 + uy;
            w2 = w2 + uz;
        }
        const float r0 = ct * w0 - st * w1, r1 = st * w0 + ct * w1;
        ux = C[0] * r0 + C[1] * r1 + C[2] * w2;
        uy = C[3] * r0 + C[4] * r1 + C[5] * w2;
        uz = C[6] * r0 + C[7] * r1 + C[8] * w2;
    }

    __device__ __forceinline__ float finish(const ChainConsts<J>& cc, const float* tgt3) const
    {
        const float px = dhc[12 * J + 0] + ux, py = dhc[12 * J + 1] + uy, pz = dhc[12 * J + 2] + uz;
        const float ex = px - tgt3[0], ey = py - tgt3[1], ez = pz - tgt3[2];
        const float distance = ((ex * ex + ey * ey) + ez * ez) * cc.eff_w[J];
        float f = distance + angle_weight<TERMS>(cc) * rot_diff;
        if constexpr (TERMS & kTermPenalty) f = f + limit_weight<TERMS>(cc) * pen;
        return f;
    }
};

template <class Topo, int MODE, int TERMS>
using TipAccFor =
    std::conditional_t<Topo::kDH, TipBackAccDH<Topo, MODE, TERMS>, TipBackAcc<Topo, MODE, TERMS>>;

// x, rest: [D]; tgt: [3J] (per node); dhc: the folded chain's constants (TopoDH);
// soft: the soft limits [lo 3J | hi 3J] (SwarmShared::soft, or cc.aux + 4J).
template <class Topo, int MODE, int TERMS>
__device__ __forceinline__ float fitness(const ChainConsts<Topo::J>& cc, const float* x, const float* rest,
                                         const float* tgt, float* node_pos /* [3J] or nullptr */,
                                         const float* dhc, const float* soft)
{
    constexpr int A = Topo::A;
    if constexpr (kTipBackward<Topo, MODE, TERMS>) {
        if (!node_pos) {
            constexpr int J = Topo::J;
            using Acc = TipAccFor<Topo, MODE, TERMS>;
            Acc tb(dhc, soft);
#pragma unroll
            for (int k = 1; k <= J; ++k) tb.angles(k, x + A * (k - 1), rest + A * (k - 1));
#pragma unroll
            for (int k = J; k >= 1; --k) tb.back(cc, k, node_trig<Acc::HW, A>(x + A * (k - 1)));
            return tb.finish(cc, tgt + 3 * (J - 1));
        }
    }
    CandBuf<Topo, TERMS> cb;
    FitnessFor<Topo, MODE, TERMS> acc(cc, dhc, soft, cb.v);
#pragma unroll
    for (int k = 1; k <= Topo::J; ++k) {
        acc.node(cc, k, x + A * (k - 1), rest + A * (k - 1), tgt + 3 * (k - 1), node_pos);
    }
    return acc.finish(cc);
}

// Sum over effectors of the Euclidean distance to target (checkDistance,
// src/Main.cpp:290-298 / src/Node.h:421-429), evaluated with the device FK
// (TERMS: the calling kernel's, for its sin/cos flavour).
template <class Topo, int MODE, int TERMS>
__device__ __forceinline__ float residual(const ChainConsts<Topo::J>& cc, const float* x, const float* tgt,
                                          const float* dhc = nullptr)
{
    constexpr int J = Topo::J;
    if constexpr (Topo::kDH) {
        FitnessAccDH<Topo, MODE, TERMS> acc(cc, dhc, cc.aux, nullptr);  // (no penalty term here)
#pragma unroll
        for (int k = 1; k <= J; ++k) acc.advance(k, x[k - 1]);
        const float dx = tgt[3 * (J - 1) + 0] - acc.px;
        const float dy = tgt[3 * (J - 1) + 1] - acc.py;
        const float dz = tgt[3 * (J - 1) + 2] - acc.pz;
        return sqrtf(dx * dx + dy * dy + dz * dz);
    } else {
        Frame F[J + 1];
        F[0] = origin_frame(cc.m0);
        float r = 0.0f;
#pragma unroll
        for (int k = 1; k <= J; ++k) {
            const int pk = Topo::kGeneric ? cc.parent[k] : Topo::parent(k);
            constexpr int HW = kHwTrig<Topo, MODE, TERMS>;
            if (kOriginFrame<Topo, TERMS> && pk == 0) {  // targets in the origin frame (kOriginFrame)
                float sa, ca, sb, cb, sc, cc_;
                sincos_fast<HW>(x[3 * (k - 1)], &sa, &ca);
                sincos_fast<HW>(x[3 * (k - 1) + 1], &sb, &cb);
                sincos_fast<HW>(x[3 * (k - 1) + 2], &sc, &cc_);
                F[k] = root_frame_sc(sa, ca, sb, cb, sc, cc_, link_len<HW>(cc, k));
            } else {
                F[k] = child_frame<MODE, false, HW>(F[pk], x[3 * (k - 1)], x[3 * (k - 1) + 1], x[3 * (k - 1) + 2],
                                                    link_len<HW>(cc, k));
            }
            if (Topo::effector(k) && cc.eff_slot[k] >= 0) {
                const float dx = tgt[3 * (k - 1) + 0] - F[k].px;
                const float dy = tgt[3 * (k - 1) + 1] - F[k].py;
                const float dz = tgt[3 * (k - 1) + 2] - F[k].pz;
                r += sqrtf(dx * dx + dy * dy + dz * dz);
            }
        }
        return r;
    }
}

// ------------------------------------------------------------ PSO update
// PSO coefficients of one solve, uniform across the workgroup.
struct PsoCoef {
    float w, c1, c2;
    float wq, c1q, c2q;  // c * 2^-32
    float wh, c1h, c2h;  // c * 2^-33
};

template <class CC>
__device__ __forceinline__ PsoCoef pso_coef(const CC& cc)
{
    return PsoCoef{cc.w, cc.c1, cc.c2, cc.wq, cc.c1q, cc.c2q, cc.wh, cc.c1h, cc.c2h};
}

// simulateParticlesKernel body for one dimension (src/kernel.cu:160-169):
//   v = w*r1*v + c1*r2*(pb - x) + c2*r3*(g - x);  x += v
// REFERENCE mode evaluates exactly that, unfused.  FAST mode folds each
// coefficient into its uniform's affine map, c*r = c*(u*2^-32 + 2^-33) =
// fma(u, c*2^-32, c*2^-33): one rounding where the reference has two (and
// three fewer multiplies per dimension).
// A draw source whose draws already carry their coefficient (the iteration
// blocks of the generator-split kernel, LdsDraws) sets kPrescaled.
template <class Rng, class = void>
struct Prescaled : std::false_type {};
template <class Rng>
struct Prescaled<Rng, std::void_t<decltype(Rng::kPrescaled)>> : std::bool_constant<Rng::kPrescaled> {};

// v = a * v + c computed into v's own register.  Left to the compiler, the FMA
// becomes a v_fmac that accumulates into c's register, so every velocity moves to
// another register each iteration and the loop's back edge pays one v_mov per
// dimension to restore the assignment (21 per wave-iteration in config 3's loop,
// 58 in config 5's, where the extra live copies also spilled).  The tied asm
// operand keeps the register.  Used by the tip-backward step (config 5: -2.6 %,
// the DH arm: -1.3 %); the software-pipelined 4-wave step keeps the compiler's
// form -- there the opaque asm costs its scheduler more than the moves (config 3
// +2 %; profiles/r04/variant_timings).
#ifndef IKPSO_INPLACE_V
#define IKPSO_INPLACE_V 1
#endif
__device__ __forceinline__ void fma_into(float& v, float a, float b, float c)  // v = a * b + c
{
#if defined(__HIP_DEVICE_COMPILE__) && IKPSO_INPLACE_V
    asm("v_fma_f32 %0, %1, %2, %3" : "+v"(v) : "v"(a), "v"(b), "v"(c));
#else
    v = __builtin_fmaf(a, b, c);
#endif
}
__device__ __forceinline__ void fma_inplace(float& v, float a, float c)  // v = a * v + c
{
#if defined(__HIP_DEVICE_COMPILE__) && IKPSO_INPLACE_V
    asm("v_fma_f32 %0, %1, %0, %2" : "+v"(v) : "v"(a), "v"(c));
#else
    v = __builtin_fmaf(a, v, c);
#endif
}

template <int MODE, bool INPLACE = false, class Rng>
__device__ __forceinline__ void pso_update(float& x, float& v, float pb, float g, const PsoCoef& k, Rng& rng)
{
    if constexpr (MODE == IKPSO_ARITH_REFERENCE && Prescaled<Rng>::value) {
        // the same operations with the first products (w * r1, c1 * r2, c2 * r3) drawn
        const float wr1 = rng.raw();
        const float c1r2 = rng.raw();
        const float c2r3 = rng.raw();
        {
#pragma clang fp contract(off)
            v = wr1 * v + c1r2 * (pb - x) + c2r3 * (g - x);
            x += v;
        }
    } else if constexpr (MODE == IKPSO_ARITH_REFERENCE) {
        const float r1 = rng.uniform();
        const float r2 = rng.uniform();
        const float r3 = rng.uniform();
        {
#pragma clang fp contract(off)
            v = k.w * r1 * v + k.c1 * r2 * (pb - x) + k.c2 * r3 * (g - x);
            x += v;
        }
    } else {
        const float a = rng.scaled(k.wq, k.wh);
        const float b = rng.scaled(k.c1q, k.c1h);
        const float c = rng.scaled(k.c2q, k.c2h);
        if constexpr (INPLACE)
            fma_inplace(v, a, __builtin_fmaf(b, pb - x, c * (g - x)));
        else
            v = __builtin_fmaf(a, v, __builtin_fmaf(b, pb - x, c * (g - x)));
        x += v;
    }
}

// FAST: the gbest-independent part of one dimension's update drawn ahead (the
// next iteration's r1, r2, r3, in the same order): pa = w r1 v + c1 r2 (pb - x),
// pc = c2 r3; the update then completes as v = pc (g - x) + pa once the new
// global best is known (pso_update_ahead).
template <class Rng>
__device__ __forceinline__ void pso_draw_ahead(float& pa, float& pc, float x, float v, float pb, const PsoCoef& k,
                                               Rng& rng)
{
    const float a = rng.scaled(k.wq, k.wh);
    const float b = rng.scaled(k.c1q, k.c1h);
    pc = rng.scaled(k.c2q, k.c2h);
    pa = __builtin_fmaf(a, v, b * (pb - x));
}
__device__ __forceinline__ void pso_update_ahead(float& x, float& v, float g, float pa, float pc)
{
    fma_into(v, pc, g - x, pa);
    x += v;
}

// clamp (src/matrix_operations.cuh:187-190)
__device__ __forceinline__ float clamp_ref(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }

// FAST mode: one v_med3_f32 (the median of v, lo, hi is the clamp for lo <= hi
// and finite v); REFERENCE mode keeps the reference's fmaxf/fminf pair, except
// in its uniform-bounds builds (BOUNDS_ORDERED: the host dispatches them only for
// finite lo <= hi, where the median is bit-identical to fminf(fmaxf(v, lo), hi)
// for every non-NaN v -- one half-rate op instead of two).
template <int MODE, bool BOUNDS_ORDERED = false>
__device__ __forceinline__ float clamp_mode(float v, float lo, float hi)
{
    if constexpr (MODE == IKPSO_ARITH_FAST || BOUNDS_ORDERED) return __builtin_amdgcn_fmed3f(v, lo, hi);
    return clamp_ref(v, lo, hi);
}

// ------------------------------------------------------------- reductions
// Order-preserving map of an fp32 value to uint32 (-0 canonicalised to +0) so
// that an unsigned min is a float min; ties then break to the lowest index,
// as thrust::min_element does.
__device__ __forceinline__ uint32_t ordered_key(float f)
{
    const uint32_t u = __float_as_uint(f + 0.0f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float key_to_float(uint32_t k)
{
    const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}

// Wave64 unsigned min, result uniform: DPP within each 16-lane row
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then the
// four row minima through readlane on the scalar unit.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x)
{
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0xB1, 0xF, 0xF, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x4E, 0xF, 0xF, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x141, 0xF, 0xF, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x140, 0xF, 0xF, false));
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 0);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 16);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 32);
    const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
    return min(min(r0, r1), min(r2, r3));
}

// Lowest lane whose key equals the (uniform) wave minimum.
__device__ __forceinline__ int wave_first_lane_eq(uint32_t key, uint32_t wmin)
{
    const uint64_t m = __ballot(key == wmin);
    return (int)__builtin_ctzll(m);
}

__device__ __forceinline__ float uniform_f32(float v)
{
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

}  // namespace ikpso
