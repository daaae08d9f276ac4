// Issue rate of dependent VALU chains against waves per SIMD on gfx950: how
// much instruction-level parallelism a wave needs to keep the SIMD issuing at
// 1, 2 and 4 waves per SIMD (the long-chain cooperative kernel runs 2).
// 256-lane workgroups (one wave per SIMD); the dynamic LDS request limits a CU
// to W workgroups, so W = waves per SIMD.  CH independent chains per lane of
// one instruction form (v_fma_f32; v_sin_f32; v_lshlrev_b32; the XORWOW step).
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/ilp_probe tools/probes/ilp_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define UNR 32

template <int OP, int CH>
__global__ void __launch_bounds__(256) k_chain(float* out, int iters, float sa, float sb)
{
    extern __shared__ float lds[];
    const float va = sa + threadIdx.x * 1e-9f, vb = sb + threadIdx.x * 1e-9f;
    float f[CH];
    unsigned u[CH][6];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        f[c] = threadIdx.x * 1e-3f + c;
#pragma unroll
        for (int k = 0; k < 6; ++k) u[c][k] = threadIdx.x * 747796405u + c * 13 + k * 2891336453u;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < UNR; ++r)
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if constexpr (OP == 0) f[c] = __builtin_fmaf(f[c], va, vb);
                if constexpr (OP == 1) f[c] = __builtin_amdgcn_sinf(f[c]);
                if constexpr (OP == 2) asm volatile("v_lshlrev_b32 %0, 4, %0" : "+v"(u[c][0]));
                if constexpr (OP == 3) {  // one XORWOW step + conversion (the generator's form)
                    const unsigned t = u[c][1] ^ (u[c][1] >> 2);
                    u[c][1] = u[c][2]; u[c][2] = u[c][3]; u[c][3] = u[c][4];
                    u[c][4] = __builtin_amdgcn_bitop3_b32(u[c][4], u[c][4] << 4, t, 0x96) ^ (t << 1);
                    u[c][0] += 362437u;
                    f[c] += __builtin_fmaf((float)(u[c][4] + u[c][0]), 2.3283064e-10f, 1.16415322e-10f);
                }
            }
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += f[c] + __uint_as_float(u[c][0] & 0x3fffffffu) + __uint_as_float(u[c][4] & 0x3fffffffu);
    if (threadIdx.x == 0) lds[0] = s;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + lds[0] * 0.0f;
}

static const char* kOp[] = {"v_fma_f32 chain", "v_sin_f32 chain", "v_lshlrev_b32 chain", "xorwow step"};
static const int kInstr[] = {1, 1, 1, 9};  // VALU instructions per step (xorwow: shifts, xors, add, add3, cvt, fma, add)

template <int OP, int CH>
static void run(int cus, int waves, void* out)
{
    const int iters = 400;
    const int blocks = cus * waves;
    const size_t lds = (160 * 1024) / waves - 1024;
    hipFuncSetAttribute((const void*)k_chain<OP, CH>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_chain<OP, CH><<<blocks, 256, lds>>>((float*)out, iters, 0.999f, 1e-3f);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int k = 0; k < 3; ++k) k_chain<OP, CH><<<blocks, 256, lds>>>((float*)out, iters, 0.999f, 1e-3f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 3;
    // cycles per step per wave: SIMD cycles elapsed / steps issued by one wave (2.4 GHz)
    const double steps = (double)iters * UNR * CH;
    const double cyc_per_step_per_simd = ms * 1e-3 * 2.4e9 / (steps * waves);
    printf("%-22s waves/SIMD %d  chains %d : %7.2f SIMD cycles per step (%5.2f per instruction)\n", kOp[OP], waves, CH,
           cyc_per_step_per_simd, cyc_per_step_per_simd / kInstr[OP]);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

template <int OP>
static void sweep(int cus, void* out)
{
    for (int w : {1, 2, 4}) {
        run<OP, 1>(cus, w, out);
        run<OP, 2>(cus, w, out);
        run<OP, 4>(cus, w, out);
        run<OP, 8>(cus, w, out);
    }
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    void* out;
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    sweep<0>(cus, out);
    sweep<1>(cus, out);
    sweep<2>(cus, out);
    sweep<3>(cus, out);
    hipFree(out);
    return 0;
}
