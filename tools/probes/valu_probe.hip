// Issue rate of single VALU instruction forms on gfx950: 1024-lane workgroups
// (16 waves, 4 per SIMD, 2 workgroups per CU), 8 independent chains of one
// instruction form, unrolled.  Reports lane-instructions/s against 78.6 T/s
// (256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz: a wave64 op every 2 cycles per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

#define CH 8
#define UNR 16

// OP: the instruction form under test (the asm of each is checked with make-asm)
template <int OP>
__global__ void __launch_bounds__(1024) k_op(float* out, int iters, float sa, float sb)
{
    const float va = sa + threadIdx.x * 1e-9f, vb = sb + threadIdx.x * 1e-9f;
    const unsigned ua = __float_as_uint(va), ub = __float_as_uint(vb);
    float f[CH];
    unsigned u[CH];
    double g[CH];
    const double da = va, db = vb;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        f[c] = threadIdx.x * 1e-3f + c;
        u[c] = threadIdx.x * 747796405u + c;
        g[c] = threadIdx.x * 1e-3 + c;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < UNR; ++r)
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if constexpr (OP == 0) f[c] = f[c] * va;                          // v_mul_f32 v,v
                if constexpr (OP == 1) f[c] = f[c] * sa;                          // v_mul_f32 v,s
                if constexpr (OP == 2) f[c] = f[c] * 0.999f;                      // v_mul_f32 literal
                if constexpr (OP == 3) f[c] = f[c] * 0.5f;                        // v_mul_f32 inline const
                if constexpr (OP == 4) f[c] = __builtin_fmaf(va, vb, f[c]);       // v_fmac_f32 v,v
                if constexpr (OP == 5) f[c] = __builtin_fmaf(f[c], va, vb);       // v_fma_f32 v,v,v
                if constexpr (OP == 6) f[c] = __builtin_fmaf(f[c], sa, sb);       // v_fma_f32 v,s,s
                if constexpr (OP == 7) f[c] = __builtin_fmaf(f[c], va, 0.999f);   // v_fmaak literal
                if constexpr (OP == 8) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[c]) : "v"(ua));
                if constexpr (OP == 9) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(u[c]));
                if constexpr (OP == 10) u[c] = __builtin_amdgcn_bitop3_b32(u[c], ua, ub, 0x96);  // bitop3 v,v,v
                if constexpr (OP == 11) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(u[c]) : "v"(ua), "v"(ub));
                if constexpr (OP == 12) asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(f[c]) : "v"(u[c]));
                if constexpr (OP == 13) f[c] = __builtin_amdgcn_fmed3f(f[c], va, vb);  // v_med3_f32
                if constexpr (OP == 14) asm volatile("v_lshrrev_b32 %0, 2, %0" : "+v"(u[c]));
                if constexpr (OP == 15) asm volatile("v_lshlrev_b32 %0, 4, %0" : "+v"(u[c]));
                if constexpr (OP == 16) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(u[c]));
                if constexpr (OP == 17) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(u[c]));
                if constexpr (OP == 18) asm volatile("v_add_u32 %0, %0, %0" : "+v"(u[c]));
                if constexpr (OP == 19) asm volatile("v_add_u32 %0, 0x587c5, %0" : "+v"(u[c]));
                if constexpr (OP == 20) asm volatile("v_alignbit_b32 %0, %0, 0, 28" : "+v"(u[c]));
                if constexpr (OP == 21) asm volatile("v_lshl_add_u32 %0, %0, 4, 0" : "+v"(u[c]));
                if constexpr (OP == 22) asm volatile("v_lshl_or_b32 %0, %0, 4, 0" : "+v"(u[c]));
                if constexpr (OP == 23) asm volatile("v_bfe_i32 %0, %0, 0, 1" : "+v"(u[c]));
                if constexpr (OP == 24) asm volatile("v_and_b32 %0, 0x80000001, %0" : "+v"(u[c]));
                if constexpr (OP == 25) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(f[c]) : "v"(va));
                if constexpr (OP == 26) asm volatile("v_max_f32 %0, %0, %1" : "+v"(f[c]) : "v"(va));
                if constexpr (OP == 27) asm volatile("v_mov_b32 %0, %1" : "=v"(u[c]) : "v"(ua));
                if constexpr (OP == 28) asm volatile("v_fmamk_f32 %0, %0, 0x3f7fbe77, %1" : "+v"(f[c]) : "v"(va));
                if constexpr (OP == 29) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(u[c]) : "v"(ub));
                if constexpr (OP == 30) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[c]) : "v"(ua));
                if constexpr (OP == 31) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(u[c]) : "v"(ua), "v"(ub));
                if constexpr (OP == 32) asm volatile("v_cvt_f32_u32_e64 %0, %1" : "=v"(f[c]) : "v"(u[c]));
                if constexpr (OP == 33) f[c] = __builtin_amdgcn_sinf(f[c]);       // v_sin_f32 (transcendental)
                if constexpr (OP == 34) {                                          // half v_sin, half v_fma:
                    if (c & 1) f[c] = __builtin_fmaf(f[c], va, vb);                // does TRANS overlap VALU?
                    else f[c] = __builtin_amdgcn_sinf(f[c]);
                }
                if constexpr (OP == 35) f[c] = __builtin_amdgcn_cosf(f[c]);       // v_cos_f32
                // fp64 and packed forms (the REFERENCE kernels' sincos runs in fp64)
                if constexpr (OP == 36) g[c] = __builtin_fma(g[c], da, db);       // v_fma_f64 v,v,v
                if constexpr (OP == 37) g[c] = g[c] * da;                         // v_mul_f64
                if constexpr (OP == 38) asm volatile("v_add_f64 %0, %0, %1" : "+v"(g[c]) : "v"(da));
                if constexpr (OP == 39) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(g[c]) : "v"(f[c]));
                if constexpr (OP == 40) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[c]) : "v"(g[c]));
                if constexpr (OP == 41) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(g[c]) : "v"(da));
                if constexpr (OP == 42) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(g[c]) : "v"(da), "v"(db));
                if constexpr (OP == 43) asm volatile("v_rndne_f32 %0, %0" : "+v"(f[c]));
                if constexpr (OP == 44) asm volatile("v_min_f32 %0, %0, %1" : "+v"(f[c]) : "v"(va));
                if constexpr (OP == 45) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[c]) : "v"(ua));
            }
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += f[c] + __uint_as_float(u[c] & 0x3fffffffu) + (float)g[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static const char* kNames[] = {
    "v_mul_f32 v,v", "v_mul_f32 v,s", "v_mul_f32 v,literal", "v_mul_f32 v,inline", "v_fmac_f32 v,v",
    "v_fma_f32 v,v,v", "v_fma_f32 v,s,s", "v_fmaak_f32 literal", "v_xor_b32 v,v", "v_lshlrev_b32 inline",
    "v_bitop3_b32 v,v,v", "v_add3_u32 v,v,v", "v_cvt_f32_u32 v", "v_med3_f32 v,v,v",
    "v_lshrrev_b32 inline", "v_lshlrev_b32 inline 4", "v_lshlrev_b32 inline 1", "v_lshrrev_b32 inline 3", "v_add_u32 v,v (x+x)", "v_add_u32 literal", "v_alignbit_b32 v,0,28 (x<<4)", "v_lshl_add_u32 v,4,0", "v_lshl_or_b32 v,4,0", "v_bfe_i32 v,0,1", "v_and_b32 literal", "v_sub_f32 v,v", "v_max_f32 v,v", "v_mov_b32 v", "v_fmamk_f32 literal", "v_lshlrev_b32 v,v (vgpr amount)", "v_add_u32 v,v,v", "v_xad_u32 v,v,v", "v_cvt_f32_u32 e64", "v_sin_f32 v", "v_sin_f32 / v_fma_f32 1:1", "v_cos_f32 v",
    "v_fma_f64 v,v,v", "v_mul_f64 v,v", "v_add_f64 v,v", "v_cvt_f64_f32", "v_cvt_f32_f64", "v_pk_mul_f32 v,v",
    "v_pk_fma_f32 v,v,v", "v_rndne_f32", "v_min_f32 v,v", "v_cndmask_b32 v,v,vcc"};


template <int OP>
static void run(int blocks, void* out)
{
    const int iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_op<OP><<<blocks, 1024>>>((float*)out, iters, 0.999f, 1e-3f);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int k = 0; k < 5; ++k) k_op<OP><<<blocks, 1024>>>((float*)out, iters, 0.999f, 1e-3f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double r = (double)blocks * 1024 * iters * UNR * CH / (ms * 1e-3);
    printf("%-32s %8.3f ms  %6.2f T lane-instr/s  %5.1f%% of 78.6  (%.2f cycles per wave64 op per SIMD)\n", kNames[OP],
           ms, r * 1e-12, r / 78.6e12 * 100, 2.0 * 78.6e12 / r);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

template <int... OPS>
static void run_all(int blocks, void* out, std::integer_sequence<int, OPS...>)
{
    (run<OPS>(blocks, out), ...);
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;
    void* out;
    hipMalloc(&out, (size_t)blocks * 1024 * 4);
    run_all(blocks, out, std::make_integer_sequence<int, 46>{});
    hipFree(out);
    return 0;
}
