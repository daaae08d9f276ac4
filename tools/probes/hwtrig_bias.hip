// The transcendental unit's sin/cos on revolutions (v_sin_f32 / v_cos_f32, FAST's
// kTrigHwRev) against fp64 sin(2 pi x) / cos(2 pi x) on 2^24 + 1 evenly spaced x in
// [-1/2, 1/2] (config 5's +-pi clamp) and every float in [0, 1/2]: the error's size,
// its mean, and its projection on (sin, cos) -- an amplitude error shows as the sin
// component of e_s, a phase error as its cos component.
//   hipcc --offload-arch=gfx950 -O2 hwtrig_bias.hip -o hwtrig_bias && ./hwtrig_bias
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_hw(const float* x, float* s, float* c, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        s[i] = __builtin_amdgcn_sinf(x[i]);
        c[i] = __builtin_amdgcn_cosf(x[i]);
    }
}

static void report(const char* name, const std::vector<float>& x, const std::vector<float>& s,
                   const std::vector<float>& c)
{
    const double tp = 6.283185307179586476925;
    double maxs = 0, maxc = 0, ms = 0, mc = 0, ss = 0, sc = 0, cs = 0, cc = 0, s2 = 0, c2 = 0, amp = 0;
    long ulp_s = 0, ulp_c = 0, n = (long)x.size();
    for (long i = 0; i < n; ++i) {
        const double sd = sin(tp * x[i]), cd = cos(tp * x[i]);
        const double es = s[i] - sd, ec = c[i] - cd;
        maxs = fmax(maxs, fabs(es));
        maxc = fmax(maxc, fabs(ec));
        ms += es, mc += ec;
        ss += es * sd, sc += es * cd, cs += ec * sd, cc += ec * cd;  // projections
        s2 += sd * sd, c2 += cd * cd;
        amp += (double)s[i] * s[i] + (double)c[i] * c[i] - 1.0;
        ulp_s += (float)sd != s[i], ulp_c += (float)cd != c[i];
    }
    printf("%s: n=%ld  max|e_sin| %.3e max|e_cos| %.3e  mean e_sin %.2e mean e_cos %.2e  "
           "e_sin ~ %.2e sin %+.2e cos, e_cos ~ %+.2e sin %.2e cos  mean(s^2+c^2-1) %.2e  "
           "not correctly rounded: sin %.3f cos %.3f\n",
           name, n, maxs, maxc, ms / n, mc / n, ss / s2, sc / c2, cs / s2, cc / c2, amp / n, (double)ulp_s / n,
           (double)ulp_c / n);
}

static void run(const char* name, std::vector<float> x)
{
    const int n = (int)x.size();
    float *dx, *ds, *dc;
    hipMalloc(&dx, n * 4);
    hipMalloc(&ds, n * 4);
    hipMalloc(&dc, n * 4);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_hw, dim3((n + 255) / 256), dim3(256), 0, 0, dx, ds, dc, n);
    std::vector<float> s(n), c(n);
    hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
    hipFree(dx), hipFree(ds), hipFree(dc);
    report(name, x, s, c);
}

// mean relative amplitude error sqrt(s^2 + c^2) - 1 over the angles (radians,
// float32) of a file, as the FAST kernels evaluate them: x * (1 / 2pi) in fp32
static void run_file(const char* path)
{
    FILE* f = fopen(path, "rb");
    if (!f) return;
    std::vector<float> x;
    float v;
    while (fread(&v, 4, 1, f) == 1) x.push_back(v * 0.159154943091895336f);
    fclose(f);
    const int n = (int)x.size();
    float *dx, *ds, *dc;
    hipMalloc(&dx, n * 4);
    hipMalloc(&ds, n * 4);
    hipMalloc(&dc, n * 4);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_hw, dim3((n + 255) / 256), dim3(256), 0, 0, dx, ds, dc, n);
    std::vector<float> s(n), c(n);
    hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
    hipFree(dx), hipFree(ds), hipFree(dc);
    double amp = 0;
    for (int i = 0; i < n; ++i) amp += sqrt((double)s[i] * s[i] + (double)c[i] * c[i]) - 1.0;
    printf("%s: n=%d  mean amplitude error %.3e\n", path, n, amp / n);
    report(path, x, s, c);
}

int main(int argc, char** argv)
{
    for (int i = 1; i < argc; ++i) run_file(argv[i]);
    if (argc > 1) return 0;
    const int N = 1 << 24;
    std::vector<float> x(N + 1);
    for (int i = 0; i <= N; ++i) x[i] = (float)(-0.5 + (double)i / N);
    run("evenly spaced [-1/2, 1/2]", x);
    std::vector<float> y;
    for (float v = 0x1p-20f; v <= 0.5f; v = nextafterf(v, 1.0f)) y.push_back(v);
    run("every float in [2^-20, 1/2]", y);
    return 0;
}
