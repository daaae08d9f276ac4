// Accuracy of candidate fp32 sincos formulations on gfx950 vs the correctly
// rounded value (computed on the device in fp64), plus v_bitop3 semantics.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cmath>
#include "ikpso_device.h"

__device__ inline void sincos_v2(float x, float* so, float* co)
{
    const float k = __builtin_rintf(x * 0.636619772367581343f);
    const int q = (int)k;
    float r = __builtin_fmaf(-k, 1.57079637050628662109375f, x);
    r = __builtin_fmaf(-k, -4.37113900018624283e-8f, r);
    r = __builtin_fmaf(-k, -1.71512451000591571e-15f, r);
    const float z = r * r;
    const float sp = __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    const float sv = __builtin_fmaf(sp * z, r, r);
    float cp = __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    cp = __builtin_fmaf(cp, z, -0.5f);
    const float cv = __builtin_fmaf(cp, z, 1.0f);
    const bool swap = q & 1;
    const float s1 = swap ? cv : sv, c1 = swap ? sv : cv;
    const unsigned t = (unsigned)q << 30;
    *so = __uint_as_float(__builtin_amdgcn_bitop3_b32(__float_as_uint(s1), t, 0x80000000u, 0x78));
    *co = __uint_as_float(__builtin_amdgcn_bitop3_b32(__float_as_uint(c1), t + 0x40000000u, 0x80000000u, 0x78));
}

__device__ inline void sincos_v3(float x, float* so, float* co)
{
    const float k = __builtin_rintf(x * 0.636619772367581343f);
    const int q = (int)k;
    float r = __builtin_fmaf(-k, 1.57079637050628662109375f, x);
    r = __builtin_fmaf(-k, -4.37113900018624283e-8f, r);
    const float z = r * r;
    const float sp = __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    const float sv = __builtin_fmaf(sp * z, r, r);
    float cp = __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    cp = __builtin_fmaf(cp, z, -0.5f);
    const float cv = __builtin_fmaf(cp, z, 1.0f);
    const bool swap = q & 1;
    const float s1 = swap ? cv : sv, c1 = swap ? sv : cv;
    const unsigned t = (unsigned)q << 30;
    *so = __uint_as_float(__builtin_amdgcn_bitop3_b32(__float_as_uint(s1), t, 0x80000000u, 0x78));
    *co = __uint_as_float(__builtin_amdgcn_bitop3_b32(__float_as_uint(c1), t + 0x40000000u, 0x80000000u, 0x78));
}

__device__ inline int ulps(float a, float b)
{
    int ia = __float_as_int(a), ib = __float_as_int(b);
    if ((ia < 0) != (ib < 0)) return a == b ? 0 : 1 << 30;
    return ia > ib ? ia - ib : ib - ia;
}

#define NV 6
struct Stats { unsigned long long bad[NV]; unsigned maxulp[NV]; float maxabs[NV]; };

__global__ void probe(float lo, float hi, unsigned long long n, unsigned seed, Stats* st, unsigned* bop_bad)
{
    __shared__ unsigned long long sbad[NV];
    __shared__ unsigned smax[NV];
    __shared__ float sabs[NV];
    if (threadIdx.x < NV) { sbad[threadIdx.x] = 0; smax[threadIdx.x] = 0; sabs[threadIdx.x] = 0; }
    __syncthreads();
    unsigned long long bad[NV] = {};
    unsigned mu[NV] = {};
    float ma[NV] = {};
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
        const float x = lo + (hi - lo) * ((h >> 8) * (1.0f / 16777216.0f));
        const float ts = (float)sin((double)x), tc = (float)cos((double)x);
        float s[NV], c[NV];
        ikpso::sincos_fast(x, &s[0], &c[0]);
        s[1] = __sinf(x); c[1] = __cosf(x);
        sincos_v2(x, &s[2], &c[2]);
        sincos_v3(x, &s[3], &c[3]);
        {   // hardware v_sin/v_cos on x / 2pi (revolutions), no range reduction
            const float t = x * 0.159154943091895336f;
            s[4] = __builtin_amdgcn_sinf(t); c[4] = __builtin_amdgcn_cosf(t);
            const float tf = __builtin_amdgcn_fractf(t);  // with v_fract_f32 first
            s[5] = __builtin_amdgcn_sinf(tf); c[5] = __builtin_amdgcn_cosf(tf);
        }
        for (int v = 0; v < NV; ++v) {
            if (s[v] != ts || c[v] != tc) bad[v]++;
            const float ea = fmaxf(fabsf(s[v] - ts), fabsf(c[v] - tc));
            ma[v] = fmaxf(ma[v], ea);
            unsigned u = 0;
            if (fabsf(ts) > 1e-3f) u = max(u, (unsigned)ulps(s[v], ts));
            if (fabsf(tc) > 1e-3f) u = max(u, (unsigned)ulps(c[v], tc));
            mu[v] = max(mu[v], u);
        }
        // bitop3 LUT checks: 0x96 = a^b^c, 0x78 = a^(b&c)
        const unsigned a = h, b = h * 747796405u + 1u, cc = b ^ (b >> 7);
        if (__builtin_amdgcn_bitop3_b32(a, b, cc, 0x96) != (a ^ b ^ cc)) atomicAdd(bop_bad, 1u);
        if (__builtin_amdgcn_bitop3_b32(a, b, cc, 0x78) != (a ^ (b & cc))) atomicAdd(bop_bad + 1, 1u);
    }
    for (int v = 0; v < NV; ++v) {
        atomicAdd(&sbad[v], bad[v]);
        atomicMax(&smax[v], mu[v]);
        atomicMax((int*)&sabs[v], __float_as_int(ma[v]));
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        atomicAdd(&st->bad[threadIdx.x], sbad[threadIdx.x]);
        atomicMax(&st->maxulp[threadIdx.x], smax[threadIdx.x]);
        atomicMax((int*)&st->maxabs[threadIdx.x], __float_as_int(sabs[threadIdx.x]));
    }
}

int main()
{
    const char* names[NV] = {"sincos_fast (current FAST)", "__sinf/__cosf", "sincos_v2 (bitop3 signs)",
                             "sincos_v3 (2-fma reduction)", "v_sin/v_cos(x/2pi)", "v_sin/v_cos(fract(x/2pi))"};
    // the last two: the FAST kernels' v_sin/v_cos range bound (kHwTrigMaxAbs, 100 rad) and the unit's own
    // +-256 revolutions
    const float ranges[6][2] = {{-7.0f, 7.0f},     {0.0f, 6.2831855f},   {-3.1415927f, 3.1415927f},
                                {-100.0f, 100.0f}, {-400.0f, 400.0f}, {-1600.0f, 1600.0f}};
    Stats* st; unsigned* bb;
    hipMalloc(&st, sizeof(Stats)); hipMalloc(&bb, 8);
    for (auto& r : ranges) {
        hipMemset(st, 0, sizeof(Stats)); hipMemset(bb, 0, 8);
        const unsigned long long n = 1ull << 26;
        hipLaunchKernelGGL(probe, dim3(4096), dim3(256), 0, 0, r[0], r[1], n, 12345u, st, bb);
        Stats h; unsigned hb[2];
        hipMemcpy(&h, st, sizeof h, hipMemcpyDeviceToHost); hipMemcpy(hb, bb, 8, hipMemcpyDeviceToHost);
        printf("x in [%g, %g], %llu samples; bitop3 mismatches xor3=%u a^(b&c)=%u\n", r[0], r[1], n, hb[0], hb[1]);
        for (int v = 0; v < NV; ++v)
            printf("  %-32s not-correctly-rounded %6.3f%%  max ulp %u  max abs %.3g\n", names[v],
                   100.0 * h.bad[v] / n, h.maxulp[v], h.maxabs[v]);
    }
    return 0;
}
