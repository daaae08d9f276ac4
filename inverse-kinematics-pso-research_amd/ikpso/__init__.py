"""ikpso -- MI355X-native PSO inverse-kinematics solver (host side).

The compute path is the gfx950 HIP library ``_lib/libikpso.so`` behind the C
ABI in ``include/ikpso.h``; this package is its Python host mirror of the
reference's solver interface (initGenerators / calculatePSO) plus the batched
multi-swarm API and the scene model on the caller's side of the boundary.
"""
from ._abi import (ARITH_FAST, ARITH_REFERENCE, COLLIDER_DTYPE, NODE, NODE_DTYPE, NODE_EFFECTOR, NODE_ORIGIN,
                   RNG_DTYPE, IkpsoError, StaleLibraryError, build_id, load)
from .scene import (RESET_TARGETS, EffectorNode, Node, OriginNode, Scene, TargetNode, check_distance,
                    init_colliders, reference_scene, serial_chain)
from .solver import (MAIN_FITNESS, MAIN_PSO, BatchSolver, FitnessConfig, PSOConfig, calculate_pso,
                     init_generators, init_generators_seeded, make_collider, particles_tensor, rng_tensor)
from .dh import DHArm, dh_arm, dh_forward
from .workloads import Workload, workload

__all__ = [
    "ARITH_FAST", "ARITH_REFERENCE", "COLLIDER_DTYPE", "init_colliders", "make_collider", "NODE", "NODE_DTYPE", "NODE_EFFECTOR", "NODE_ORIGIN", "RNG_DTYPE",
    "IkpsoError", "StaleLibraryError", "build_id", "load", "RESET_TARGETS", "EffectorNode", "Node", "OriginNode", "Scene", "TargetNode",
    "check_distance", "reference_scene", "serial_chain", "MAIN_FITNESS", "MAIN_PSO", "BatchSolver",
    "FitnessConfig", "PSOConfig", "calculate_pso", "init_generators", "init_generators_seeded",
    "particles_tensor", "rng_tensor", "Workload", "workload", "DHArm", "dh_arm", "dh_forward",
]
