/*
 * ikpso_compat.h -- the reference's own solver entry points, for a drop-in
 * link of the unchanged visualiser (src/Main.cpp) against libikpso.so.
 *
 *   initGenerators  replaces src/utility_kernels.cuh:33-47 (declared src/Main.cpp:28)
 *   calculatePSO    replaces src/kernel.cu:279-327        (declared src/Main.cpp:29)
 *
 * Same names, same parameter lists, same C++ linkage (so the mangled symbols
 * Main.cpp references resolve), same semantics: the caller allocates every
 * buffer, randoms persist across calls, the call is synchronous on return and
 * a non-zero status aborts the caller's frame loop.  The status type is
 * hipError_t (cudaError_t after the cuda->hip aliasing in INTEGRATION.md).
 *
 * Types: by default this header defines NodeCUDA, Coordinates, PSOConfig,
 * FitnessConfig, obj/obj_t and curandStateXORWOW/curandState_t with the
 * reference's layouts (src/Particle.h, src/BoxCollider.h, cuRAND).  A caller
 * that keeps including the reference's Particle.h / BoxCollider.h defines
 * IKPSO_COMPAT_REFERENCE_TYPES before including this header.
 */
#ifndef IKPSO_COMPAT_H
#define IKPSO_COMPAT_H

#include <hip/hip_runtime.h>

#ifndef DEGREES_OF_FREEDOM
#define DEGREES_OF_FREEDOM 21 /* src/ik_constants.h:3 */
#endif

/* cuRAND XORWOW state layout (48 bytes); filled by initGenerators only. */
struct curandStateXORWOW {
    unsigned int d, v[5];
    int boxmuller_flag;
    int boxmuller_flag_double;
    float boxmuller_extra;
    double boxmuller_extra_double;
};
typedef struct curandStateXORWOW curandState_t;

#ifndef IKPSO_COMPAT_REFERENCE_TYPES
enum NodeType { originNode, effectorNode, node };

struct NodeCUDA {
    NodeType nodeType;
    int parentIndex;
    float effectorWeight;
    float3 position;
    float3 rotation;
    float3 maxRotation;
    float3 minRotation;
    float length;
    float3 targetPosition;
    float3 targetRotation;
};

struct Coordinates {
    float positions[DEGREES_OF_FREEDOM];
};

struct FitnessConfig {
    float angleWeight;
    float distanceWeight;
    float errorThreshold;
    FitnessConfig(float angleWeight = 3.0f, float distanceWeight = 0.0f, float errorThreshold = 0.1f)
        : angleWeight(angleWeight), distanceWeight(distanceWeight), errorThreshold(errorThreshold) {}
};

struct PSOConfig {
    float _inertia;
    float _local;
    float _global;
    int _iterations;
    PSOConfig(float inertia = 0.2f, float local = 0.5f, float global = 0.7f, int iterations = 10)
        : _inertia(inertia), _local(local), _global(global), _iterations(iterations) {}
};

struct obj {
    float x, y, z;
    float3 pos;
    float4 quat;
};
typedef struct obj obj_t;
#endif /* IKPSO_COMPAT_REFERENCE_TYPES */

/* The caller's DEGREES_OF_FREEDOM, seen by the library (which is built for one
 * value, -DDEGREES_OF_FREEDOM=N): calculatePSO reads `chain` and `result` with
 * its own D, so a caller built with another D gets hipErrorInvalidValue
 * instead of a silently wrong node count.  A weak definition in every caller
 * translation unit that includes this header (the library's own build does
 * not define it); a caller that never includes it is not checked. */
#ifndef IKPSO_BUILDING_LIBRARY
extern "C" __attribute__((weak, visibility("default"))) const int ikpso_compat_caller_dof = DEGREES_OF_FREEDOM;
#endif

hipError_t initGenerators(curandState_t* randoms, int size);
hipError_t calculatePSO(float* particles, float* positions, float* bests, curandState_t* randoms, int size,
                        NodeCUDA* chain, PSOConfig psoConfig, FitnessConfig fitConfig, Coordinates* result,
                        obj_t* colliders, int colliderCount);

#endif /* IKPSO_COMPAT_H */
