"""ctypes binding of the C ABI declared in include/ikpso.h.

The shared library ``_lib/libikpso.so`` is built in-tree by
``csrc/Makefile`` (``__graft_entry__.build()``).  There is no fallback: if the
library is missing every entry point raises, so a GPU run can never silently
fall back to a CPU implementation.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

LIB_DIR = Path(__file__).resolve().parent / "_lib"
LIB_PATH = LIB_DIR / "libikpso.so"

# ---------------------------------------------------------------- constants
IKPSO_OK = 0
IKPSO_ERR_INVALID_ARG = 1
IKPSO_ERR_UNSUPPORTED = 2
IKPSO_ERR_HIP = 3
IKPSO_ERR_NO_MEMORY = 4

NODE_ORIGIN, NODE_EFFECTOR, NODE = 0, 1, 2  # src/Particle.h:10-15

ARITH_FAST = 0
ARITH_REFERENCE = 1

KERNEL_AUTO = 0
KERNEL_RESIDENT = 1
KERNEL_STREAMING = 2
KERNEL_COOP = 3

# ------------------------------------------------------------ numpy layouts
#: NodeCUDA (src/Particle.h:24-39), 88 bytes.
NODE_DTYPE = np.dtype(
    [
        ("node_type", "<i4"),
        ("parent_index", "<i4"),
        ("effector_weight", "<f4"),
        ("position", "<f4", (3,)),
        ("rotation", "<f4", (3,)),
        ("max_rotation", "<f4", (3,)),
        ("min_rotation", "<f4", (3,)),
        ("length", "<f4"),
        ("target_position", "<f4", (3,)),
        ("target_rotation", "<f4", (3,)),
    ]
)
assert NODE_DTYPE.itemsize == 88

#: curandStateXORWOW layout, 48 bytes.
RNG_DTYPE = np.dtype(
    [
        ("d", "<u4"),
        ("v", "<u4", (5,)),
        ("boxmuller_flag", "<i4"),
        ("boxmuller_flag_double", "<i4"),
        ("boxmuller_extra", "<f4"),
        ("pad_", "<u4"),
        ("boxmuller_extra_double", "<f8"),
    ]
)
assert RNG_DTYPE.itemsize == 48
RNG_WORDS = 12  # int32 words per state

#: obj_t (src/BoxCollider.h:4-10), 48 bytes: edge lengths x, y, z; centre; quaternion (x, y, z, w).
COLLIDER_DTYPE = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("pos", "<f4", (3,)), ("pad_", "<f4", (2,)), ("quat", "<f4", (4,))]
)
assert COLLIDER_DTYPE.itemsize == 48

ABI_VERSION = 5

FLAG_POSREF_NODE_SLOT = 1  # IKPSO_FLAG_POSREF_NODE_SLOT
FLAG_NO_FOLD = 2  # IKPSO_FLAG_NO_FOLD


# ------------------------------------------------------------ ctypes structs
class PSOConfig(ctypes.Structure):
    """PSOConfig (src/Particle.h:70-85), passed by value."""

    _fields_ = [
        ("inertia", ctypes.c_float),
        ("local", ctypes.c_float),
        ("global_", ctypes.c_float),
        ("iterations", ctypes.c_int32),
    ]


class FitnessConfig(ctypes.Structure):
    """FitnessConfig (src/Particle.h:55-68), passed by value."""

    _fields_ = [
        ("angle_weight", ctypes.c_float),
        ("distance_weight", ctypes.c_float),
        ("error_threshold", ctypes.c_float),
    ]


class SolverDesc(ctypes.Structure):
    _fields_ = [
        ("chain", ctypes.c_void_p),
        ("node_count", ctypes.c_int32),
        ("particles", ctypes.c_int32),
        ("pso", PSOConfig),
        ("fit", FitnessConfig),
        ("arith", ctypes.c_int32),
        ("kernel", ctypes.c_int32),
        ("positions", ctypes.c_void_p),
        ("limit_weight", ctypes.c_float),
        ("reserved1", ctypes.c_float),
        ("soft_lo", ctypes.c_void_p),
        ("soft_hi", ctypes.c_void_p),
        ("colliders", ctypes.c_void_p),
        ("collider_count", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("axis_mask", ctypes.c_void_p),  # ABI >= 4
    ]


assert ctypes.sizeof(PSOConfig) == 16
assert ctypes.sizeof(FitnessConfig) == 12

# Every symbol include/ikpso.h declares: name -> (restype, argtypes)
_vp, _i32, _i64, _u64, _f = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
SIGNATURES = {
    "ikpso_init_generators": (_i32, [_vp, ctypes.c_int, _vp]),
    "ikpso_init_generators_seeded": (_i32, [_vp, _i64, _u64, _vp]),
    "ikpso_calculate_pso": (
        _i32,
        [_vp, _vp, _vp, _vp, ctypes.c_int, _vp, ctypes.c_int, PSOConfig, FitnessConfig, _vp, _vp, ctypes.c_int, _vp],
    ),
    "ikpso_solver_create": (_i32, [ctypes.POINTER(SolverDesc), ctypes.POINTER(_vp)]),
    "ikpso_solver_destroy": (_i32, [_vp]),
    "ikpso_solver_seed": (_i32, [_vp, _i64, _u64, _i64, _vp]),
    "ikpso_solve_batch": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp]),
    "ikpso_solver_sync": (_i32, [_vp]),
    "ikpso_solver_fallbacks": (_i64, [_vp]),
    "ikpso_coop_fallbacks": (_i64, []),
    "ikpso_solver_evaluate": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "ikpso_solver_generator_states": (_i32, [_vp, _i64, _i64, _vp, _vp]),
    "ikpso_solver_dof": (ctypes.c_int, [_vp]),
    "ikpso_solver_effectors": (ctypes.c_int, [_vp]),
    "ikpso_solver_collider_count": (ctypes.c_int, [_vp]),
    "ikpso_solver_kernel_name": (ctypes.c_char_p, [_vp]),
    "ikpso_abi_version": (ctypes.c_int, []),
    "ikpso_status_string": (ctypes.c_char_p, [_i32]),
    "ikpso_last_hip_error": (ctypes.c_int, []),
    "ikpso_build_id": (ctypes.c_char_p, []),
}

_LIB = None


class IkpsoError(RuntimeError):
    def __init__(self, status: int, where: str):
        lib = load()
        msg = lib.ikpso_status_string(status).decode()
        hip = lib.ikpso_last_hip_error() if status == IKPSO_ERR_HIP else 0
        super().__init__(f"{where}: {msg} (status {status}{', hipError ' + str(hip) if hip else ''})")
        self.status = status


class StaleLibraryError(RuntimeError):
    """libikpso.so was built from other sources than the tree it is loaded from."""


def build_id() -> str:
    """The loaded library's source hash (``ikpso_build_id``)."""
    return load().ikpso_build_id().decode()


def load() -> ctypes.CDLL:
    """Load libikpso.so (RTLD_GLOBAL not needed).  Raises if it is missing, has
    another ABI version, or was built from other sources than this tree
    (``ikpso_build_id`` vs ``_buildid.tree_id()``; IKPSO_ALLOW_STALE=1 accepts
    it, for variant builds loaded through IKPSO_LIB)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = Path(os.environ.get("IKPSO_LIB", LIB_PATH))
    if not path.exists():
        raise FileNotFoundError(
            f"{path} not found: build the HIP library first (python -c 'import __graft_entry__ as g; g.build()' "
            "or make -C inverse-kinematics-pso-research_amd/csrc)"
        )
    lib = ctypes.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ikpso_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{path}: ABI version {lib.ikpso_abi_version()}, expected {ABI_VERSION} (rebuild)")
    from . import _buildid

    built, tree = lib.ikpso_build_id().decode(), _buildid.tree_id()
    if tree is not None and built != tree and os.environ.get("IKPSO_ALLOW_STALE") != "1":
        raise StaleLibraryError(
            f"{path} was built from sources {built}, this tree is {tree}: rebuild (make -C "
            "inverse-kinematics-pso-research_amd/csrc), or set IKPSO_ALLOW_STALE=1 for a variant build")
    _LIB = lib
    return lib


def check(status: int, where: str) -> None:
    if status != IKPSO_OK:
        raise IkpsoError(status, where)
