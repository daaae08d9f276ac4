/* batch_c.c -- the batched C ABI (include/ikpso.h) from plain C: B independent
 * IK targets for the reference arm (src/Main.cpp:76-116), one launch.
 * HIP's C runtime API for device memory; no torch, no Python.
 * usage: batch_c [B] [iterations] [colliders]
 *   colliders: the reference's initColliders boxes 0 and 3 (src/Main.cpp:537-559) and a
 *   third box out of the arm's reach (the collider term, its host-side early-out) */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ikpso.h"

#define CHECK_HIP(x)                                                                   \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            return 1;                                                                  \
        }                                                                              \
    } while (0)
#define CHECK_IK(x)                                                                          \
    do {                                                                                     \
        ikpso_status s_ = (x);                                                               \
        if (s_ != IKPSO_OK) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, ikpso_status_string(s_));      \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

static void reference_arm(ikpso_node* n)
{
    static const int parent[8] = {-1, 0, 1, 2, 3, 4, 4, 4};
    static const float rest[8][3] = {{0, 0, 0},     {0, 1.57f, 0}, {0, 1.57f, 0}, {0, 1.57f, 0},
                                     {0, 1.57f, 0}, {0, 1.57f, 0}, {0, 0, 1.57f}, {0, 0, 1.57f}};
    static const float reset[3][3] = {{0.75f, 1, -2.5f}, {-0.75f, 1, -2.5f}, {0, 0, -2.5f}};
    const float two_pi = 2.0f * 3.14159265358979323846f;
    memset(n, 0, sizeof(ikpso_node) * 8);
    for (int k = 0; k < 8; ++k) {
        n[k].node_type = k == 0 ? IKPSO_NODE_ORIGIN : (k >= 5 ? IKPSO_NODE_EFFECTOR : IKPSO_NODE);
        n[k].parent_index = parent[k];
        n[k].effector_weight = k >= 5 ? 1.0f : 0.0f;
        for (int c = 0; c < 3; ++c) {
            n[k].rotation[c] = rest[k][c];
            n[k].max_rotation[c] = two_pi;
            if (k >= 5) n[k].target_position[c] = reset[k - 5][c];
        }
        n[k].length = k == 0 ? 0.0f : 1.0f;
    }
}

int main(int argc, char** argv)
{
    const int B = argc > 1 ? atoi(argv[1]) : 256;
    const int iters = argc > 2 ? atoi(argv[2]) : 500;
    const int P = 1024, D = 21, E = 3;
    ikpso_node chain[8];
    reference_arm(chain);

    /* targets: the reset targets + a deterministic offset per swarm */
    float* h_tg = (float*)malloc(sizeof(float) * B * E * 3);
    for (int b = 0; b < B; ++b)
        for (int e = 0; e < E; ++e)
            for (int c = 0; c < 3; ++c)
                h_tg[(b * E + e) * 3 + c] = chain[5 + e].target_position[c] + 0.25f * sinf(0.7f * b + 1.3f * e + c);
    float *d_tg, *d_ang, *d_fit, *d_res;
    CHECK_HIP(hipMalloc((void**)&d_tg, sizeof(float) * B * E * 3));
    CHECK_HIP(hipMalloc((void**)&d_ang, sizeof(float) * B * D));
    CHECK_HIP(hipMalloc((void**)&d_fit, sizeof(float) * B));
    CHECK_HIP(hipMalloc((void**)&d_res, sizeof(float) * B));
    CHECK_HIP(hipMemcpy(d_tg, h_tg, sizeof(float) * B * E * 3, hipMemcpyHostToDevice));

    ikpso_solver_desc desc;
    memset(&desc, 0, sizeof(desc));
    desc.chain = chain;
    desc.node_count = 8;
    desc.particles = P;
    desc.pso.inertia = 0.5f;
    desc.pso.local = 0.5f;
    desc.pso.global = 1.25f;
    desc.pso.iterations = iters;
    desc.fit.angle_weight = 3.0f;
    desc.fit.error_threshold = 0.1f;
    ikpso_collider boxes[3];
    memset(boxes, 0, sizeof(boxes));
    if (argc > 3 && strcmp(argv[3], "colliders") == 0) {
        static const float pos[3][3] = {{1.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 1.0f}, {40.0f, 0.0f, 0.0f}};
        for (int i = 0; i < 3; ++i) {
            boxes[i].x = boxes[i].y = boxes[i].z = 1.0f;
            for (int c = 0; c < 3; ++c) boxes[i].pos[c] = pos[i][c];
            boxes[i].quat[3] = 1.0f;
        }
        desc.colliders = boxes;
        desc.collider_count = 3;
    }
    ikpso_solver* s;
    CHECK_IK(ikpso_solver_create(&desc, &s));
    CHECK_IK(ikpso_solver_seed(s, B, 0, 0, NULL));
    CHECK_IK(ikpso_solve_batch(s, d_tg, NULL, B, iters, d_ang, d_fit, d_res, NULL));  /* warm-up */
    hipEvent_t a, z;
    CHECK_HIP(hipEventCreate(&a));
    CHECK_HIP(hipEventCreate(&z));
    CHECK_HIP(hipEventRecord(a, NULL));
    CHECK_IK(ikpso_solve_batch(s, d_tg, NULL, B, iters, d_ang, d_fit, d_res, NULL));
    CHECK_HIP(hipEventRecord(z, NULL));
    CHECK_HIP(hipEventSynchronize(z));
    float ms = 0.0f;
    CHECK_HIP(hipEventElapsedTime(&ms, a, z));

    float* h_fit = (float*)malloc(sizeof(float) * B);
    float* h_res = (float*)malloc(sizeof(float) * B);
    CHECK_HIP(hipMemcpy(h_fit, d_fit, sizeof(float) * B, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(h_res, d_res, sizeof(float) * B, hipMemcpyDeviceToHost));
    double mf = 0, mr = 0;
    int finite = 1;
    for (int b = 0; b < B; ++b) {
        mf += h_fit[b];
        mr += h_res[b];
        finite &= isfinite(h_fit[b]) && isfinite(h_res[b]);
    }
    printf("kernel %s: %d swarms x %d particles x %d iterations in %.3f ms = %.3e particle-updates/s\n",
           ikpso_solver_kernel_name(s), B, P, iters, ms, (double)B * P * iters / (ms * 1e-3));
    printf("mean fitness %.6f, mean residual %.6f, finite %d, colliders tested %d\n", mf / B, mr / B, finite,
           ikpso_solver_collider_count(s));
    ikpso_solver_destroy(s);
    return finite ? 0 : 2;
}
