// Every float x with |x| < 4096 (both signs: 2 x 0x45800000 bit patterns, zeros and
// subnormals included) through the device sincos routines of ikpso_device.h, compiled
// for the host: REFERENCE (sincos_reference) compared bit for bit with the CPU
// oracle's sinf/cosf, (float)sin((double)x) / (float)cos((double)x)
// (oracle/ikpso_oracle.c); FAST's polynomial (sincos_fast<kTrigPoly>, the collider
// kernels' and wide-range chains' sin/cos) by its largest absolute error and its
// largest ulp error where |value| >= 2^-10.  Prints one JSON line.
// Test infrastructure: tests/test_sincos_exhaustive.py.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "ikpso_device.h"

static uint32_t bits_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static long ulp_dist(float a, float b)
{
    int32_t ia = (int32_t)bits_of(a), ib = (int32_t)bits_of(b);
    if (ia < 0) ia = (int32_t)0x80000000 - ia;  // monotone integer line through +-0
    if (ib < 0) ib = (int32_t)0x80000000 - ib;
    return labs((long)ia - (long)ib);
}

struct Acc {
    long n = 0, sin_bad = 0, cos_bad = 0, fast_ulp = 0;
    double fast_abs = 0.0;
    uint32_t first_bad[8] = {};
    int nbad = 0;
};

int main(int argc, char** argv)
{
    const uint32_t top = 0x45800000u;  // bit pattern of 4096.0f
    int nt = argc > 1 ? atoi(argv[1]) : (int)std::thread::hardware_concurrency();
    const bool fast = argc > 2 && atoi(argv[2]) != 0;  // also FAST's polynomial (about 3x the time)
    if (nt < 1) nt = 1;
    std::vector<Acc> acc(nt);
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            Acc& a = acc[t];
            for (uint64_t u = t; u < 2ull * top; u += nt) {  // interleaved: large |x| costs libm more
                const uint32_t b = u < top ? (uint32_t)u : (0x80000000u | (uint32_t)(u - top));
                float x;
                memcpy(&x, &b, 4);
                float s, c, fs, fc;
                ikpso::sincos_reference(x, &s, &c);
                const double sd = sin((double)x), cd = cos((double)x);
                const float ts = (float)sd, tc = (float)cd;
                const bool sb = bits_of(s) != bits_of(ts), cb = bits_of(c) != bits_of(tc);
                a.sin_bad += sb;
                a.cos_bad += cb;
                if ((sb || cb) && a.nbad < 8) a.first_bad[a.nbad++] = b;
                ++a.n;
                if (!fast) continue;
                ikpso::sincos_fast<ikpso::kTrigPoly>(x, &fs, &fc);
                const double es = fabs((double)fs - sd), ec = fabs((double)fc - cd);
                if (es > a.fast_abs) a.fast_abs = es;
                if (ec > a.fast_abs) a.fast_abs = ec;
                if (fabsf(ts) >= 0x1p-10f) { long d = ulp_dist(fs, ts); if (d > a.fast_ulp) a.fast_ulp = d; }
                if (fabsf(tc) >= 0x1p-10f) { long d = ulp_dist(fc, tc); if (d > a.fast_ulp) a.fast_ulp = d; }
            }
        });
    for (auto& x : th) x.join();
    Acc tot;
    printf("{\"floats\": ");
    for (auto& a : acc) {
        tot.n += a.n; tot.sin_bad += a.sin_bad; tot.cos_bad += a.cos_bad;
        if (a.fast_abs > tot.fast_abs) tot.fast_abs = a.fast_abs;
        if (a.fast_ulp > tot.fast_ulp) tot.fast_ulp = a.fast_ulp;
    }
    printf("%ld, \"domain\": \"|x| < 4096, every float\", \"threads\": %d, \"reference_sin_mismatch\": %ld, "
           "\"reference_cos_mismatch\": %ld, ", tot.n, nt, tot.sin_bad, tot.cos_bad);
    if (fast) printf("\"fast_poly_max_abs\": %.3e, \"fast_poly_max_ulp\": %ld, ", tot.fast_abs, tot.fast_ulp);
    printf("\"first_mismatch\": [");
    int k = 0;
    for (auto& a : acc)
        for (int i = 0; i < a.nbad && k < 8; ++i, ++k) printf("%s\"%08x\"", k ? ", " : "", a.first_bad[i]);
    printf("]}\n");
    return 0;
}
