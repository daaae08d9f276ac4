"""Python mirror of the reference's solver interface over the C ABI.

Reference entry points (src/ = InverseKinematicsResearch/InverseKinematicsResearch/):
    initGenerators(curandState_t* randoms, int size)        src/utility_kernels.cuh:33-47
    calculatePSO(particles, positions, bests, randoms, size, chain, PSOConfig,
                 FitnessConfig, Coordinates* result, obj_t* colliders,
                 int colliderCount)                          src/kernel.cu:279-327
Both return a status code (cudaError_t there, ikpso_status here: 0 = success,
anything else = the caller's frame loop aborts, src/Main.cpp:225-226).

Device buffers are torch tensors on a ROCm device (torch is plumbing for
device memory and streams); host-side buffers may be numpy arrays.  The
batched API (``BatchSolver``) is the MI355X-native extension: B independent
swarms per call, one kernel launch.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from . import _abi
from ._abi import NODE_DTYPE, RNG_WORDS, FitnessConfig as _CFit, PSOConfig as _CPso, SolverDesc


@dataclass
class PSOConfig:
    """PSOConfig (src/Particle.h:70-85); defaults are the struct's own.
    The visualiser uses PSOConfig(0.5, 0.5, 1.25, 15) (src/Main.cpp:130)."""

    inertia: float = 0.2
    local: float = 0.5
    global_: float = 0.7
    iterations: int = 10

    def c(self) -> _CPso:
        return _CPso(self.inertia, self.local, self.global_, int(self.iterations))


@dataclass
class FitnessConfig:
    """FitnessConfig (src/Particle.h:55-68); the visualiser uses (3, 0, 0.1)."""

    angle_weight: float = 3.0
    distance_weight: float = 0.0
    error_threshold: float = 0.1

    def c(self) -> _CFit:
        return _CFit(self.angle_weight, self.distance_weight, self.error_threshold)


MAIN_PSO = PSOConfig(0.5, 0.5, 1.25, 15)       # src/Main.cpp:130
MAIN_FITNESS = FitnessConfig(3.0, 0.0, 0.1)    # src/Main.cpp:131


def _torch():
    import torch

    return torch


def _dev_ptr(t) -> Optional[int]:
    """Device pointer of a torch tensor (must be on a GPU and contiguous)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("expected a device tensor")
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    return t.data_ptr()


def _any_ptr(x, keep: list) -> Optional[int]:
    """Pointer to host (numpy) or device (torch) memory."""
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        a = np.ascontiguousarray(x)
        keep.append(a)
        return a.ctypes.data
    if x.is_cuda:
        return _dev_ptr(x)
    if not x.is_contiguous():
        x = x.contiguous()
    keep.append(x)
    return x.data_ptr()


def _stream_handle(stream) -> Optional[int]:
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream or None


def _colliders(colliders) -> np.ndarray:
    """obj_t array (COLLIDER_DTYPE) from a compatible numpy array."""
    b = np.ascontiguousarray(colliders)
    if b.dtype != _abi.COLLIDER_DTYPE:
        if b.dtype.itemsize != _abi.COLLIDER_DTYPE.itemsize:
            raise TypeError("colliders must be an obj_t (COLLIDER_DTYPE) array")
        b = b.view(_abi.COLLIDER_DTYPE)
    return b.reshape(-1)


def make_collider(size, pos, quat=(0.0, 0.0, 0.0, 1.0)) -> np.ndarray:
    """One obj_t: size = (x, y, z) box edge lengths, pos = centre, quat = (x, y, z, w)."""
    c = np.zeros(1, dtype=_abi.COLLIDER_DTYPE)
    c["x"], c["y"], c["z"] = size
    c["pos"] = pos
    c["quat"] = quat
    return c


def rng_tensor(count: int, device="cuda"):
    """Device buffer for `count` generator states (48 bytes each, curandState_t layout)."""
    torch = _torch()
    return torch.zeros((count, RNG_WORDS), dtype=torch.int32, device=device)


def particles_tensor(size: int, dof: int, device="cuda"):
    """Device buffer for the reference's particles array: [3][dof][size] floats."""
    torch = _torch()
    return torch.zeros((3, dof, size), dtype=torch.float32, device=device)


def init_generators(randoms, size: int, stream=None) -> int:
    """initGenerators: randoms[i] = curand_init(i, 0, 0).  Returns the status."""
    lib = _abi.load()
    return lib.ikpso_init_generators(_dev_ptr(randoms), int(size), _stream_handle(stream))


def init_generators_seeded(randoms, count: int, seed_base: int, stream=None) -> int:
    lib = _abi.load()
    return lib.ikpso_init_generators_seeded(_dev_ptr(randoms), int(count), int(seed_base), _stream_handle(stream))


def calculate_pso(particles, positions, bests, randoms, size: int, chain: np.ndarray, pso_config: PSOConfig,
                  fit_config: FitnessConfig, result, colliders=None, collider_count: int = 0, stream=None) -> int:
    """calculatePSO over the C ABI; same arguments, same meaning, same status
    convention.  `chain` is a NODE_DTYPE array (host) or device tensor;
    `result` receives the global-best angles (numpy array or tensor);
    `colliders` an obj_t array (numpy COLLIDER_DTYPE or a device tensor) with
    `collider_count` entries (src/kernel.cu:104-136)."""
    lib = _abi.load()
    keep: list = []
    if isinstance(colliders, np.ndarray):
        colliders = _colliders(colliders)
    if isinstance(chain, np.ndarray):
        if chain.dtype != NODE_DTYPE:
            raise TypeError("chain must be an ikpso NODE_DTYPE array")
        node_count = int(chain.shape[0])
    else:
        node_count = int(chain.numel() * chain.element_size() // NODE_DTYPE.itemsize)
    return lib.ikpso_calculate_pso(
        _dev_ptr(particles), _any_ptr(positions, keep), _dev_ptr(bests), _dev_ptr(randoms), int(size),
        _any_ptr(chain, keep), node_count, pso_config.c(), fit_config.c(), _any_ptr(result, keep),
        _any_ptr(colliders, keep), int(collider_count), _stream_handle(stream))


class BatchSolver:
    """B independent swarms (IK targets) per call over one shared chain.

    RNG streams are owned by the solver and persist across calls (like the
    reference's randoms buffer); local swarm b of a solver seeded with
    first_swarm = f draws the streams curand_init(seed_base + (f + b) * P + i).
    """

    def __init__(self, chain: np.ndarray, particles: int, pso: PSOConfig = MAIN_PSO,
                 fit: FitnessConfig = MAIN_FITNESS, arith: str = "fast", positions=None,
                 limit_weight: float = 0.0, soft_lo=None, soft_hi=None, kernel: str = "auto", colliders=None,
                 posref_node_slot: bool = False, axis_mask=None, fold: bool = True):
        self._lib = _abi.load()
        if chain.dtype != NODE_DTYPE:
            raise TypeError("chain must be an ikpso NODE_DTYPE array")
        self.chain = np.ascontiguousarray(chain)
        self.P = int(particles)
        self.pso = pso
        self.fit = fit
        keep: list = []
        desc = SolverDesc()
        desc.chain = self.chain.ctypes.data
        desc.node_count = self.chain.shape[0]
        desc.particles = self.P
        desc.pso = pso.c()
        desc.fit = fit.c()
        desc.arith = {"fast": _abi.ARITH_FAST, "reference": _abi.ARITH_REFERENCE}[arith]
        desc.kernel = {"auto": _abi.KERNEL_AUTO, "resident": _abi.KERNEL_RESIDENT,
                       "streaming": _abi.KERNEL_STREAMING, "coop": _abi.KERNEL_COOP}[kernel]
        desc.positions = _any_ptr(None if positions is None else np.asarray(positions, np.float32), keep)
        desc.limit_weight = float(limit_weight)
        desc.soft_lo = _any_ptr(None if soft_lo is None else np.asarray(soft_lo, np.float32), keep)
        desc.soft_hi = _any_ptr(None if soft_hi is None else np.asarray(soft_hi, np.float32), keep)
        desc.flags = (_abi.FLAG_POSREF_NODE_SLOT if posref_node_slot else 0) | (0 if fold else _abi.FLAG_NO_FOLD)
        if axis_mask is not None:  # [node_count] uint8: bit c = Euler angle c of node k is free
            m = np.ascontiguousarray(axis_mask, dtype=np.uint8)
            if m.shape != (self.chain.shape[0],):
                raise ValueError(f"axis_mask must have one entry per node ({self.chain.shape[0]})")
            desc.axis_mask = _any_ptr(m, keep)
        self.axis_mask = None if axis_mask is None else np.array(axis_mask, dtype=np.uint8)
        if colliders is not None and len(colliders):
            boxes = _colliders(colliders)
            desc.colliders = _any_ptr(boxes, keep)
            desc.collider_count = int(boxes.shape[0])
        handle = ctypes.c_void_p()
        _abi.check(self._lib.ikpso_solver_create(ctypes.byref(desc), ctypes.byref(handle)), "ikpso_solver_create")
        self._h = handle
        self.dof = self._lib.ikpso_solver_dof(self._h)
        self.effectors = self._lib.ikpso_solver_effectors(self._h)
        self.capacity = 0

    @property
    def collider_count(self) -> int:
        """Colliders the kernels test (0 when none is within the arm's reach)."""
        return self._lib.ikpso_solver_collider_count(self._h)

    @property
    def kernel(self) -> str:
        """Kernel variant the solver dispatches to (the last solve's, once one ran)."""
        return self._lib.ikpso_solver_kernel_name(self._h).decode()

    def seed(self, capacity: int, seed_base: int = 0, first_swarm: int = 0, stream=None) -> None:
        torch = _torch()
        _abi.check(self._lib.ikpso_solver_seed(self._h, int(capacity), int(seed_base), int(first_swarm),
                                               _stream_handle(stream)), "ikpso_solver_seed")
        self._device = torch.device("cuda", torch.cuda.current_device())  # where the generator states live
        self.capacity = max(self.capacity, int(capacity))

    def _check_tensor(self, t, name: str, device) -> None:
        """float32, contiguous, on the solver's device (the kernels read raw fp32)."""
        torch = _torch()
        if t is None:
            return
        if not t.is_cuda or t.device != device:
            raise ValueError(f"{name} must be on {device}, got {t.device}")
        if t.dtype != torch.float32:
            raise ValueError(f"{name} must be float32, got {t.dtype}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")

    def solve(self, targets=None, start_pose=None, iterations: Optional[int] = None, num_swarms: Optional[int] = None,
              out: Optional[Tuple] = None, residual: bool = True, stream=None, sync: bool = True):
        """targets: device [B, E, 3] (None: chain targets); start_pose: device [B, D] or None.
        Returns (angles [B, D], fitness [B], residual [B] or None) device tensors.
        sync: settle a cooperative-family solve before returning (ikpso_solver_sync:
        waits for it, and re-runs it on the streaming kernels if the GPU's other work
        kept a group from assembling); no effect on the other families, which stay
        stream-ordered and asynchronous."""
        torch = _torch()
        if num_swarms is None:
            if targets is None:
                raise ValueError("num_swarms is required when targets is None")
            num_swarms = int(targets.shape[0])
        B = int(num_swarms)
        it = self.pso.iterations if iterations is None else int(iterations)
        if targets is not None and tuple(targets.shape) != (B, self.effectors, 3):
            raise ValueError(f"targets must be [{B}, {self.effectors}, 3]")
        if start_pose is not None and tuple(start_pose.shape) != (B, self.dof):
            raise ValueError(f"start_pose must be [{B}, {self.dof}]")
        dev = getattr(self, "_device", None) or torch.device("cuda", torch.cuda.current_device())
        if out is None:
            angles = torch.empty((B, self.dof), dtype=torch.float32, device=dev)
            fitness = torch.empty((B,), dtype=torch.float32, device=dev)
            res = torch.empty((B,), dtype=torch.float32, device=dev) if residual else None
        else:
            angles, fitness, res = out
            if tuple(angles.shape) != (B, self.dof) or tuple(fitness.shape) != (B,) or (
                    res is not None and tuple(res.shape) != (B,)):
                raise ValueError("out must be ([B, D], [B], [B] or None)")
        for t, name in ((targets, "targets"), (start_pose, "start_pose"), (angles, "out angles"),
                        (fitness, "out fitness"), (res, "out residual")):
            self._check_tensor(t, name, dev)
        _abi.check(self._lib.ikpso_solve_batch(self._h, _dev_ptr(targets), _dev_ptr(start_pose), B, it,
                                               _dev_ptr(angles), _dev_ptr(fitness), _dev_ptr(res),
                                               _stream_handle(stream)), "ikpso_solve_batch")
        if sync:
            _abi.check(self._lib.ikpso_solver_sync(self._h), "ikpso_solver_sync")
        return angles, fitness, res

    def sync(self) -> None:
        """ikpso_solver_sync: settle the last solve (see solve(sync=...))."""
        _abi.check(self._lib.ikpso_solver_sync(self._h), "ikpso_solver_sync")

    @property
    def fallbacks(self) -> int:
        """Cooperative solves of this solver that were re-run on the streaming kernels."""
        return int(self._lib.ikpso_solver_fallbacks(self._h))

    def generator_states(self, first_swarm: int = 0, count: Optional[int] = None, stream=None) -> np.ndarray:
        """The solver-owned generator states of local swarms [first_swarm, first_swarm + count):
        int32 words [count * P, 12] (curandState layout, swarm-major), after settling a
        pending solve (ikpso_solver_generator_states)."""
        n = (self.capacity - int(first_swarm)) if count is None else int(count)
        out = np.zeros((n * self.P, RNG_WORDS), dtype=np.int32)
        _abi.check(self._lib.ikpso_solver_generator_states(self._h, int(first_swarm), n, out.ctypes.data,
                                                           _stream_handle(stream)), "ikpso_solver_generator_states")
        return out

    def evaluate(self, angles, targets=None, rest=None, stream=None):
        """Device FK + fitness for angle vectors [n, D]: (fitness [n], node positions [n, J, 3])."""
        torch = _torch()
        n = int(angles.shape[0])
        if tuple(angles.shape) != (n, self.dof):
            raise ValueError(f"angles must be [n, {self.dof}]")
        for t, name in ((angles, "angles"), (targets, "targets"), (rest, "rest")):
            self._check_tensor(t, name, angles.device)
        fit = torch.empty((n,), dtype=torch.float32, device=angles.device)
        pos = torch.empty((n, self.chain.shape[0] - 1, 3), dtype=torch.float32, device=angles.device)
        _abi.check(self._lib.ikpso_solver_evaluate(self._h, _dev_ptr(angles), _dev_ptr(targets), _dev_ptr(rest), n,
                                                   _dev_ptr(fit), _dev_ptr(pos), _stream_handle(stream)),
                   "ikpso_solver_evaluate")
        return fit, pos

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.ikpso_solver_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
