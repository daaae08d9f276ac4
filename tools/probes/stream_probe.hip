// Achievable HBM rate of the streaming kernel's access pattern: per particle
// read 3 planes and write 2 planes of D floats (x, v, pbest -> x, v), with
// 4-B-per-lane accesses ([plane][d][P], lane = particle) vs 16-B-per-lane
// accesses ([plane][d/4][P][4]).  Prints GB/s of algorithmic bytes.
// build: hipcc --offload-arch=gfx950 -O3 stream_probe.hip -o stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int D = 60;

__global__ void __launch_bounds__(256) k_dword(float* s, long P)
{
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i >= P) return;
    float* x = s;
    float* v = s + (long)D * P;
    const float* pb = s + 2L * D * P;
#pragma unroll 4
    for (int d = 0; d < D; ++d) {
        const float xv = x[d * P + i], vv = v[d * P + i], pv = pb[d * P + i];
        const float nv = 0.5f * vv + 0.25f * (pv - xv);
        v[d * P + i] = nv;
        x[d * P + i] = xv + nv;
    }
}

__global__ void __launch_bounds__(256) k_quad(float4* s, long P)
{
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i >= P) return;
    constexpr int Q = D / 4;
    float4* x = s;
    float4* v = s + (long)Q * P;
    const float4* pb = s + 2L * Q * P;
#pragma unroll 3
    for (int q = 0; q < Q; ++q) {
        const float4 xv = x[q * P + i], vv = v[q * P + i], pv = pb[q * P + i];
        float4 nv, nx;
        nv.x = 0.5f * vv.x + 0.25f * (pv.x - xv.x);
        nv.y = 0.5f * vv.y + 0.25f * (pv.y - xv.y);
        nv.z = 0.5f * vv.z + 0.25f * (pv.z - xv.z);
        nv.w = 0.5f * vv.w + 0.25f * (pv.w - xv.w);
        nx.x = xv.x + nv.x;
        nx.y = xv.y + nv.y;
        nx.z = xv.z + nv.z;
        nx.w = xv.w + nv.w;
        v[q * P + i] = nv;
        x[q * P + i] = nx;
    }
}

// read-only sweep of the same 3 planes (reference rate)
__global__ void __launch_bounds__(256) k_quad_read(const float4* s, long P, float* out)
{
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i >= P) return;
    constexpr int Q = D / 4;
    float acc = 0.0f;
#pragma unroll 3
    for (int q = 0; q < 3 * Q; ++q) {
        const float4 a = s[q * P + i];
        acc += a.x + a.y + a.z + a.w;
    }
    if (acc == 12345.0f) out[0] = acc;
}

int main()
{
    const long P = 8L << 20;  // 8M particles: 3 planes x 60 x 4 B = 6 GB
    float* s;
    if (hipMalloc(&s, sizeof(float) * 3L * D * P) != hipSuccess) return 1;
    float* out;
    (void)hipMalloc(&out, 4);
    (void)hipMemset(s, 0, sizeof(float) * 3L * D * P);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const dim3 grid((unsigned)((P + 255) / 256));
    for (int rep = 0; rep < 3; ++rep) {
        float ms;
        hipLaunchKernelGGL(k_dword, grid, dim3(256), 0, 0, s, P);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_dword, grid, dim3(256), 0, 0, s, P);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
        const double bytes = 5.0 * D * 4 * P;
        printf("dword  r3w2: %.3f ms  %.0f GB/s\n", ms, bytes / ms / 1e6);
        hipLaunchKernelGGL(k_quad, grid, dim3(256), 0, 0, (float4*)s, P);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_quad, grid, dim3(256), 0, 0, (float4*)s, P);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
        printf("quad   r3w2: %.3f ms  %.0f GB/s\n", ms, bytes / ms / 1e6);
        hipLaunchKernelGGL(k_quad_read, grid, dim3(256), 0, 0, (const float4*)s, P, out);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_quad_read, grid, dim3(256), 0, 0, (const float4*)s, P, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
        printf("quad   read: %.3f ms  %.0f GB/s\n", ms, 3.0 * D * 4 * P / ms / 1e6);
    }
    return 0;
}
