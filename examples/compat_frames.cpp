// compat_frames.cpp -- the reference visualiser's solve loop (src/Main.cpp:
// 120-250, src/ = InverseKinematicsResearch/InverseKinematicsResearch/) with
// the window removed, linked against libikpso.so through the reference's own
// entry points (include/ikpso_compat.h): the caller code a maintainer keeps
// when swapping the CUDA solver for the MI355X one.
//
//   - buffers exactly as src/Main.cpp:137-141 allocates them (device
//     particles/bests/randoms, managed chain/positions/result/colliders);
//   - initGenerators once (:145), then per frame: ToCUDA + FillPositions
//     (:222-223), calculatePSO (:225, abort on error), FromCoords (:227);
//   - a "recorded" test case as the R key starts it: resetArm, count frames
//     until checkDistance <= 0.025 (:171-215, :290-298, :330-337).
//
// Host forward kinematics (glm in the reference, src/Node.h:92-102) is a small
// float 4x4 product here.  usage: compat_frames [cases] [N]
//
// compat_frames replay <skip> <frames> [N]: the recorded session of the
// reference's results.xlsx DEGREES_3 -- `skip` unrecorded frames, then the R key
// (resetArm) and `frames` solves with the answer fed back, each printed as
// "frame k: a0 .. a20" (%.9g round-trips float).  tests/test_gpu_examples.py
// compares frames 70-74 with the recording and the oracle's replay.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ikpso_compat.h"

namespace {

struct M4 {
    float c[16];  // row-major
};

M4 eye()
{
    M4 m{};
    for (int i = 0; i < 4; ++i) m.c[5 * i] = 1.0f;
    return m;
}

M4 mul(const M4& a, const M4& b)
{
    M4 o{};
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            float s = 0.0f;
            for (int k = 0; k < 4; ++k) s += a.c[4 * r + k] * b.c[4 * k + c];
            o.c[4 * r + c] = s;
        }
    return o;
}

M4 rot_euler(float3 a)  // rotateEuler: Rx * Ry * Rz
{
    M4 x = eye(), y = eye(), z = eye();
    x.c[5] = cosf(a.x), x.c[6] = -sinf(a.x), x.c[9] = sinf(a.x), x.c[10] = cosf(a.x);
    y.c[0] = cosf(a.y), y.c[2] = sinf(a.y), y.c[8] = -sinf(a.y), y.c[10] = cosf(a.y);
    z.c[0] = cosf(a.z), z.c[1] = -sinf(a.z), z.c[4] = sinf(a.z), z.c[5] = cosf(a.z);
    return mul(mul(x, y), z);
}

M4 translate(float tx, float ty, float tz)
{
    M4 m = eye();
    m.c[3] = tx, m.c[7] = ty, m.c[11] = tz;
    return m;
}

// The reference arm (src/Main.cpp:76-116) as the DFS-ordered node table that
// Node::ToCUDA produces: origin, 4 elbows, 3 wrist effectors on the last elbow.
const int kNodes = DEGREES_OF_FREEDOM / 3 + 1;
const float kTwoPi = 2.0f * 3.14159265358979323846f;
const float3 kRest[8] = {{0, 0, 0},     {0, 1.57f, 0}, {0, 1.57f, 0}, {0, 1.57f, 0},
                         {0, 1.57f, 0}, {0, 1.57f, 0}, {0, 0, 1.57f}, {0, 0, 1.57f}};
const float3 kReset[3] = {{0.75f, 1, -2.5f}, {-0.75f, 1, -2.5f}, {0, 0, -2.5f}};  // resetArm targets

void scene(NodeCUDA* n)
{
    const int parent[8] = {-1, 0, 1, 2, 3, 4, 4, 4};
    for (int k = 0; k < kNodes; ++k) {
        n[k] = NodeCUDA{};
        n[k].nodeType = k == 0 ? originNode : (k >= 5 ? effectorNode : node);
        n[k].parentIndex = parent[k];
        n[k].effectorWeight = k >= 5 ? 1.0f : 0.0f;
        n[k].rotation = kRest[k];
        n[k].minRotation = make_float3(0, 0, 0);
        n[k].maxRotation = make_float3(kTwoPi, kTwoPi, kTwoPi);
        n[k].length = k == 0 ? 0.0f : 1.0f;
        if (k >= 5) n[k].targetPosition = kReset[k - 5];
    }
}

void world(const NodeCUDA* n, M4* m)  // GetModelMatrix for every node
{
    m[0] = mul(translate(n[0].position.x, n[0].position.y, n[0].position.z), rot_euler(n[0].rotation));
    for (int k = 1; k < kNodes; ++k)
        m[k] = mul(m[n[k].parentIndex], mul(rot_euler(n[k].rotation), translate(n[k].length, 0, 0)));
}

float check_distance(const NodeCUDA* n)  // checkDistance: sum of effector distances
{
    M4 m[8];
    world(n, m);
    float d = 0.0f;
    for (int k = 5; k < kNodes; ++k) {
        const float dx = n[k].targetPosition.x - m[k].c[3], dy = n[k].targetPosition.y - m[k].c[7],
                    dz = n[k].targetPosition.z - m[k].c[11];
        d += sqrtf(dx * dx + dy * dy + dz * dz);
    }
    return d;
}

void fill_positions(const NodeCUDA* n, float* positions)  // FillPositions: node i -> slot i + 1
{
    M4 m[8];
    world(n, m);
    for (int k = 0; k < kNodes; ++k)
        for (int c = 0; c < 4; ++c) positions[4 * (k + 1) + c] = c == 3 ? 1.0f : m[k].c[4 * c + 3];
}

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

}  // namespace

int main(int argc, char** argv)
{
    const bool replay = argc > 1 && strcmp(argv[1], "replay") == 0;
    const int skip = replay && argc > 2 ? atoi(argv[2]) : 0;
    const int record = replay && argc > 3 ? atoi(argv[3]) : 0;
    const int cases = replay ? 0 : (argc > 1 ? atoi(argv[1]) : 5);
    const int N = argc > (replay ? 4 : 2) ? atoi(argv[replay ? 4 : 2]) : 16384;  // src/Main.cpp:17
    float *particles, *bests, *positions;
    curandState_t* randoms;
    NodeCUDA* chain;
    Coordinates* result;
    obj_t* colliders;
    CHECK(hipMalloc(&particles, sizeof(float) * N * 3 * DEGREES_OF_FREEDOM));
    CHECK(hipMalloc(&bests, sizeof(float) * N));
    CHECK(hipMalloc(&randoms, sizeof(curandState_t) * N));
    CHECK(hipMallocManaged(&chain, sizeof(NodeCUDA) * kNodes));
    CHECK(hipMallocManaged(&positions, sizeof(float) * 4 * (kNodes + 1)));
    CHECK(hipMallocManaged(&result, sizeof(Coordinates)));
    CHECK(hipMallocManaged(&colliders, sizeof(obj_t)));
    const PSOConfig pso(0.5f, 0.5f, 1.25f, 15);  // src/Main.cpp:130
    const FitnessConfig fit(3.0f, 0.0f, 0.1f);   // src/Main.cpp:131
    CHECK(initGenerators(randoms, N));

    NodeCUDA arm[8];
    scene(arm);
    auto solve = [&](int frame, bool print) -> hipError_t {
        for (int k = 0; k < kNodes; ++k) chain[k] = arm[k];  // ToCUDA
        fill_positions(arm, positions);
        const hipError_t st = calculatePSO(particles, positions, bests, randoms, N, chain, pso, fit, result,
                                           colliders, 0);
        if (st != hipSuccess) return st;
        for (int k = 1; k < kNodes; ++k)  // FromCoords
            arm[k].rotation = make_float3(result->positions[3 * (k - 1)], result->positions[3 * (k - 1) + 1],
                                          result->positions[3 * (k - 1) + 2]);
        if (print) {
            printf("frame %d:", frame);
            for (int d = 0; d < DEGREES_OF_FREEDOM; ++d) printf(" %.9g", result->positions[d]);
            printf("\n");
        }
        return hipSuccess;
    };
    if (replay) {
        for (int f = 0; f < skip + record; ++f) {
            if (f == skip) scene(arm);  // R: resetArm, src/Main.cpp:412-418
            const hipError_t st = solve(f, f >= skip);
            if (st != hipSuccess) {
                fprintf(stderr, "calculatePSO failed: %s\n", hipGetErrorString(st));
                return 2;
            }
        }
        return 0;
    }
    std::vector<int> frames;
    double solve_ms = 0.0;
    int solves = 0;
    for (int c = 0; c < cases; ++c) {
        scene(arm);  // resetArm: default pose + reset targets
        int f = 0;
        while (f < 2000) {
            ++f;
            if (check_distance(arm) <= 0.025f) break;
            for (int k = 0; k < kNodes; ++k) chain[k] = arm[k];  // ToCUDA
            fill_positions(arm, positions);
            const auto t0 = std::chrono::steady_clock::now();
            const hipError_t st = calculatePSO(particles, positions, bests, randoms, N, chain, pso, fit, result,
                                               colliders, 0);
            if (c > 0 || f > 1) {  // the first call (code-object load, first allocations) is warm-up
                solve_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                ++solves;
            }
            if (st != hipSuccess) {  // the frame loop breaks on a failed solve (src/Main.cpp:226)
                fprintf(stderr, "calculatePSO failed: %s\n", hipGetErrorString(st));
                return 2;
            }
            for (int k = 1; k < kNodes; ++k)  // FromCoords
                arm[k].rotation = make_float3(result->positions[3 * (k - 1)], result->positions[3 * (k - 1) + 1],
                                              result->positions[3 * (k - 1) + 2]);
        }
        frames.push_back(f);
    }
    printf("frames to converge:");
    for (int f : frames) printf(" %d", f);
    printf("\ncalculatePSO N=%d: %d calls, %.3f ms per call\n", N, solves, solves ? solve_ms / solves : 0.0);
    for (int f : frames)
        if (f >= 2000) return 3;
    return 0;
}
