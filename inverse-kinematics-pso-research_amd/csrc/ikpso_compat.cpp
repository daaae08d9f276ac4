// ikpso_compat.cpp -- initGenerators / calculatePSO with the reference's
// signatures (include/ikpso_compat.h), forwarding to the C ABI.
#define IKPSO_BUILDING_LIBRARY
#include "ikpso_compat.h"

#include "ikpso.h"

// Defined (weakly) by callers that include ikpso_compat.h: their DEGREES_OF_FREEDOM.
extern "C" __attribute__((weak)) const int ikpso_compat_caller_dof;

static_assert(sizeof(NodeCUDA) == sizeof(ikpso_node), "NodeCUDA layout");
static_assert(sizeof(curandState_t) == sizeof(ikpso_rng_state), "curandState_t layout");
static_assert(sizeof(obj_t) == sizeof(ikpso_collider), "obj_t layout");
static_assert(sizeof(PSOConfig) == sizeof(ikpso_pso_config), "PSOConfig layout");
static_assert(sizeof(FitnessConfig) == sizeof(ikpso_fitness_config), "FitnessConfig layout");

static hipError_t to_hip(ikpso_status s)
{
    switch (s) {
    case IKPSO_OK: return hipSuccess;
    case IKPSO_ERR_INVALID_ARG: return hipErrorInvalidValue;
    case IKPSO_ERR_UNSUPPORTED: return hipErrorNotSupported;
    case IKPSO_ERR_NO_MEMORY: return hipErrorOutOfMemory;
    default: {
        const int e = ikpso_last_hip_error();
        return e ? (hipError_t)e : hipErrorUnknown;
    }
    }
}

hipError_t initGenerators(curandState_t* randoms, int size)
{
    return to_hip(ikpso_init_generators(reinterpret_cast<ikpso_rng_state*>(randoms), size, nullptr));
}

hipError_t calculatePSO(float* particles, float* positions, float* bests, curandState_t* randoms, int size,
                        NodeCUDA* chain, PSOConfig psoConfig, FitnessConfig fitConfig, Coordinates* result,
                        obj_t* colliders, int colliderCount)
{
    // Coordinates and the node table are sized by the caller's DEGREES_OF_FREEDOM:
    // refuse a caller compiled for another chain length
    if (&ikpso_compat_caller_dof != nullptr && ikpso_compat_caller_dof != DEGREES_OF_FREEDOM)
        return hipErrorInvalidConfiguration;
    const ikpso_pso_config pso{psoConfig._inertia, psoConfig._local, psoConfig._global, psoConfig._iterations};
    const ikpso_fitness_config fit{fitConfig.angleWeight, fitConfig.distanceWeight, fitConfig.errorThreshold};
    return to_hip(ikpso_calculate_pso(particles, positions, bests, reinterpret_cast<ikpso_rng_state*>(randoms), size,
                                      reinterpret_cast<const ikpso_node*>(chain), DEGREES_OF_FREEDOM / 3 + 1, pso, fit,
                                      result->positions, reinterpret_cast<const ikpso_collider*>(colliders),
                                      colliderCount, nullptr));
}
