"""ctypes wrapper of the CPU oracle (oracle/ikpso_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline.  The product
package never imports it.  Parity status: the oracle is pinned by the
reference's own recorded data (Documentation/results.xlsx FK rows and
convergence distances, tests/golden/) and its XORWOW step by rocRAND's
xorwow_engine; the cuRAND seeding constants are spec-pinned.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "libikpso_oracle.so"

NODE_DTYPE = np.dtype(
    [
        ("node_type", "<i4"), ("parent_index", "<i4"), ("effector_weight", "<f4"), ("position", "<f4", (3,)),
        ("rotation", "<f4", (3,)), ("max_rotation", "<f4", (3,)), ("min_rotation", "<f4", (3,)),
        ("length", "<f4"), ("target_position", "<f4", (3,)), ("target_rotation", "<f4", (3,)),
    ]
)
RNG_DTYPE = np.dtype(
    [
        ("d", "<u4"), ("v", "<u4", (5,)), ("boxmuller_flag", "<i4"), ("boxmuller_flag_double", "<i4"),
        ("boxmuller_extra", "<f4"), ("pad_", "<u4"), ("boxmuller_extra_double", "<f8"),
    ]
)

# obj_t (src/BoxCollider.h:4-10): x, y, z are the box's full edge lengths.
BOX_DTYPE = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("pos", "<f4", (3,)), ("pad_", "<f4", (2,)), ("quat", "<f4", (4,))]
)

_LIB = None
_NATIVE = None
_P = ctypes.c_void_p
NATIVE_PATH = HERE / "_build" / "native" / "libikpso_oracle.so"


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def load():
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            build()
        _LIB = _bind(ctypes.CDLL(str(LIB_PATH)))
    return _LIB


def load_native():
    """The CPU-baseline build of the same source (-O3 -march=native, still
    -ffp-contract=off: same results), compiled for the host this runs on."""
    global _NATIVE
    if _NATIVE is None:
        subprocess.run(["make", "-s", "-C", str(HERE), "native"], check=True)
        _NATIVE = _bind(ctypes.CDLL(str(NATIVE_PATH)))
    return _NATIVE


FMA_PATH = HERE / "_build" / "fma" / "libikpso_oracle.so"
_FMA = None


def load_fma():
    """The same source with FMA contraction (-mfma -ffp-contract=fast): a second valid
    fp32 evaluation of every solve, one rounding apart from load()'s -- the tier-B
    envelope (tests/golden/make_tierb.py; replaces round 4's tools/tier_b_envelope.py)."""
    global _FMA
    if _FMA is None:
        subprocess.run(["make", "-s", "-C", str(HERE), "fma"], check=True)
        _FMA = _bind(ctypes.CDLL(str(FMA_PATH)))
    return _FMA


def _bind(lib):
    sig = {
        "orc_sizeof_rng": (ctypes.c_int, []),
        "orc_sizeof_node": (ctypes.c_int, []),
        "orc_curand_init": (None, [ctypes.c_uint64, _P]),
        "orc_curand": (ctypes.c_uint32, [_P]),
        "orc_curand_uniform": (ctypes.c_float, [_P]),
        "orc_init_generators": (None, [_P, ctypes.c_int64, ctypes.c_uint64]),
        "orc_uniform_stream": (None, [_P, _P, ctypes.c_int]),
        "orc_skipahead": (None, [_P, ctypes.c_int64, ctypes.c_uint64]),
        "orc_chain_matrices": (None, [_P, ctypes.c_int, _P, _P]),
        "orc_fitness": (ctypes.c_float, [_P, ctypes.c_int, _P, _P, ctypes.c_float, ctypes.c_float]),
        "orc_fitness_ex": (ctypes.c_float, [_P, ctypes.c_int, _P, _P, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_float, _P, _P, _P, ctypes.c_int]),
        "orc_sizeof_box": (ctypes.c_int, []),
        "orc_gjk_intersect": (ctypes.c_int, [_P, _P]),
        "orc_node_collides": (ctypes.c_int, [_P, _P, ctypes.c_float, _P, ctypes.c_int]),
        "orc_node_positions": (None, [_P, ctypes.c_int, _P, _P]),
        "orc_residual": (ctypes.c_float, [_P, ctypes.c_int, _P]),
        "orc_calculate_pso": (
            ctypes.c_int,
            [_P, _P, _P, _P, ctypes.c_int64, _P, ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float,
             ctypes.c_int, ctypes.c_float, ctypes.c_float, _P],
        ),
        "orc_calculate_pso_ex": (
            ctypes.c_int,
            [_P, _P, _P, _P, ctypes.c_int64, _P, ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float,
             ctypes.c_int, ctypes.c_float, ctypes.c_float, _P, ctypes.c_float, _P, _P, _P, ctypes.c_int],
        ),
        "orc_fitness_mask": (ctypes.c_float, [_P, ctypes.c_int, _P, _P, ctypes.c_float, ctypes.c_float,
                                              ctypes.c_float, _P, _P, _P, ctypes.c_int, _P]),
        "orc_solve_batch_mask": (
            ctypes.c_int,
            [_P, ctypes.c_int, _P, _P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_float,
             ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, _P, _P, _P, _P, ctypes.c_int,
             ctypes.c_float, _P, _P, _P, ctypes.c_int, _P],
        ),
        "orc_solve_batch": (
            ctypes.c_int,
            [_P, ctypes.c_int, _P, _P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_float,
             ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, _P, _P, _P, _P, ctypes.c_int,
             ctypes.c_float, _P, _P, _P, ctypes.c_int],
        ),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    assert lib.orc_sizeof_rng() == 48 and lib.orc_sizeof_node() == 88 and lib.orc_sizeof_box() == 48
    return lib


def _p(a):
    return None if a is None else a.ctypes.data


def _boxes(colliders):
    """(array or None, count) for a BOX_DTYPE-compatible collider array."""
    if colliders is None or len(colliders) == 0:
        return None, 0
    b = np.ascontiguousarray(colliders)
    b = b.view(BOX_DTYPE) if b.dtype != BOX_DTYPE else b
    return b, int(b.shape[0])


def make_box(size, pos, quat=(0.0, 0.0, 0.0, 1.0)) -> np.ndarray:
    """One obj_t: size = (x, y, z) edge lengths, quat = (x, y, z, w)."""
    b = np.zeros((), dtype=BOX_DTYPE)
    b["x"], b["y"], b["z"] = size
    b["pos"] = pos
    b["quat"] = quat
    return b


def gjk_intersect(a, b) -> bool:
    """GJKIntersect (src/kernel.cu:532-536) of two obj_t boxes."""
    a = np.ascontiguousarray(a, dtype=BOX_DTYPE)
    b = np.ascontiguousarray(b, dtype=BOX_DTYPE)
    return bool(load().orc_gjk_intersect(a.ctypes.data, b.ctypes.data))


def _chain(chain) -> np.ndarray:
    c = np.ascontiguousarray(chain)
    return c.view(NODE_DTYPE) if c.dtype != NODE_DTYPE else c


def init_generators(count: int, seed_base: int = 0) -> np.ndarray:
    st = np.zeros(count, dtype=RNG_DTYPE)
    load().orc_init_generators(_p(st), int(count), int(seed_base))
    return st


def uniform_stream(state: np.ndarray, n: int) -> np.ndarray:
    """Draw n curand_uniform values from one state (advances it in place)."""
    out = np.empty(n, dtype=np.float32)
    load().orc_uniform_stream(state.ctypes.data, _p(out), int(n))
    return out


def skipahead(states: np.ndarray, n: int) -> np.ndarray:
    """Advance every state by n draws in place (GF(2) jump; = n curand() calls)."""
    st = np.ascontiguousarray(states)
    assert st.dtype == RNG_DTYPE and st is states, "skipahead needs a contiguous RNG_DTYPE array"
    load().orc_skipahead(st.ctypes.data, int(st.shape[0]), int(n))
    return states


def raw_stream(state: np.ndarray, n: int) -> np.ndarray:
    lib = load()
    return np.array([lib.orc_curand(state.ctypes.data) for _ in range(n)], dtype=np.uint32)


def chain_matrices(chain, angles) -> np.ndarray:
    c = _chain(chain)
    a = np.ascontiguousarray(angles, dtype=np.float32)
    out = np.empty((c.shape[0], 4, 4), dtype=np.float32)
    load().orc_chain_matrices(_p(c), c.shape[0], _p(a), _p(out))
    return out


def node_positions(chain, angles) -> np.ndarray:
    c = _chain(chain)
    a = np.ascontiguousarray(angles, dtype=np.float32)
    out = np.empty((c.shape[0] - 1, 3), dtype=np.float32)
    load().orc_node_positions(_p(c), c.shape[0], _p(a), _p(out))
    return out


def _f32(x):
    return None if x is None else np.ascontiguousarray(x, dtype=np.float32)


def fitness(chain, angles, angle_weight=3.0, distance_weight=0.0, positions=None, limit_weight=0.0, soft_lo=None,
            soft_hi=None, colliders=None) -> np.float32:
    c = _chain(chain)
    a = _f32(angles)
    pos, lo, hi = _f32(positions), _f32(soft_lo), _f32(soft_hi)
    bx, nb = _boxes(colliders)
    return np.float32(load().orc_fitness_ex(_p(c), c.shape[0], _p(pos), _p(a), angle_weight, distance_weight,
                                            limit_weight, _p(lo), _p(hi), _p(bx), nb))


def _mask(axis_mask, node_count):
    if axis_mask is None:
        return None
    m = np.ascontiguousarray(axis_mask, dtype=np.uint8)
    if m.shape != (node_count,):
        raise ValueError(f"axis_mask must have one entry per node ({node_count})")
    return m


def free_dims(chain, axis_mask=None) -> np.ndarray:
    """Euler indices 3*(k-1)+c of the free dimensions of a (masked) chain."""
    c = _chain(chain)
    m = _mask(axis_mask, c.shape[0])
    return np.array([3 * (k - 1) + a for k in range(1, c.shape[0]) for a in range(3)
                     if m is None or (m[k] >> a) & 1], dtype=np.int64)


def expand(chain, angles, axis_mask=None) -> np.ndarray:
    """Full Euler vector of a masked chain from its free dimensions (locked axes at rest)."""
    c = _chain(chain)
    full = np.asarray(c["rotation"][1:], dtype=np.float32).reshape(-1).copy()
    full[free_dims(c, axis_mask)] = np.asarray(angles, dtype=np.float32)
    return full


def fitness_mask(chain, angles, axis_mask, angle_weight=3.0, distance_weight=0.0, positions=None,
                 limit_weight=0.0, soft_lo=None, soft_hi=None, colliders=None) -> np.float32:
    """calculateDistance of a masked chain; angles = its free dimensions."""
    c = _chain(chain)
    a = _f32(angles)
    pos, lo, hi = _f32(positions), _f32(soft_lo), _f32(soft_hi)
    bx, nb = _boxes(colliders)
    m = _mask(axis_mask, c.shape[0])
    return np.float32(load().orc_fitness_mask(_p(c), c.shape[0], _p(pos), _p(a), angle_weight, distance_weight,
                                              limit_weight, _p(lo), _p(hi), _p(bx), nb, _p(m)))


def residual(chain, angles) -> np.float32:
    c = _chain(chain)
    a = np.ascontiguousarray(angles, dtype=np.float32)
    return np.float32(load().orc_residual(_p(c), c.shape[0], _p(a)))


def calculate_pso(chain, size: int, randoms: np.ndarray, inertia=0.5, local=0.5, glob=1.25, iterations=15,
                  angle_weight=3.0, distance_weight=0.0, positions=None, limit_weight=0.0, soft_lo=None,
                  soft_hi=None, colliders=None):
    """One reference solve.  Advances `randoms` in place.
    Returns (result [D], particles [3, D, size], bests [size])."""
    c = _chain(chain)
    D = 3 * (c.shape[0] - 1)
    parts = np.zeros((3, D, size), dtype=np.float32)
    bests = np.zeros(size, dtype=np.float32)
    res = np.zeros(D, dtype=np.float32)
    pos = None if positions is None else np.ascontiguousarray(positions, dtype=np.float32)
    lo, hi = _f32(soft_lo), _f32(soft_hi)
    bx, nb = _boxes(colliders)
    load().orc_calculate_pso_ex(_p(parts), _p(pos), _p(bests), _p(randoms), int(size), _p(c), c.shape[0], inertia,
                                local, glob, int(iterations), angle_weight, distance_weight, _p(res), limit_weight,
                                _p(lo), _p(hi), _p(bx), nb)
    return res, parts, bests


def solve_batch(chain, targets, start_pose, particles: int, iterations: int, rng: np.ndarray, inertia=0.5,
                local=0.5, glob=1.25, angle_weight=3.0, distance_weight=0.0, positions=None, threads: int = 0,
                limit_weight=0.0, soft_lo=None, soft_hi=None, colliders=None, lib=None, axis_mask=None):
    """B independent reference solves (OpenMP over swarms).  rng: [B*P] states, advanced in place.
    lib: the loaded oracle to run (default load(); load_native() for the CPU baseline).
    axis_mask: [node_count] uint8, bit c = Euler angle c of node k is free (None: all; the
    reference); D = the free dimensions, start_pose / angles / soft limits over those.
    Returns (angles [B, D], fitness [B], residual [B])."""
    c = _chain(chain)
    m = _mask(axis_mask, c.shape[0])
    D = len(free_dims(c, m))
    t = np.ascontiguousarray(targets, dtype=np.float32)
    B = t.shape[0]
    sp = None if start_pose is None else np.ascontiguousarray(start_pose, dtype=np.float32)
    pos = None if positions is None else np.ascontiguousarray(positions, dtype=np.float32)
    ang = np.zeros((B, D), dtype=np.float32)
    fit = np.zeros(B, dtype=np.float32)
    res = np.zeros(B, dtype=np.float32)
    lo, hi = _f32(soft_lo), _f32(soft_hi)
    bx, nb = _boxes(colliders)
    err = (lib or load()).orc_solve_batch_mask(
        _p(c), c.shape[0], _p(t), _p(sp), B, int(particles), int(iterations), inertia, local, glob, angle_weight,
        distance_weight, _p(pos), _p(rng), _p(ang), _p(fit), _p(res), int(threads), limit_weight, _p(lo), _p(hi),
        _p(bx), nb, _p(m))
    if err:
        raise RuntimeError(f"orc_solve_batch failed ({err})")
    return ang, fit, res
