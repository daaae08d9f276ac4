"""BASELINE.json configurations as concrete, seeded inputs.

    1  reference scene, reset targets, P=256,  I=200, B=1      (CPU plumbing)
    2  reference scene, reset targets, P=1024, I=500, B=1      (1 GPU, latency)
    3  reset targets + U[-0.25,0.25]^3 per effector, P=1024, I=500, B=4096 (1 GPU)
    4  as 3 with B=65536 sharded over the ranks
    5  20-joint serial chain (D=60), tip effector, targets in a 2-4 shell,
       soft joint-limit penalty lambda=10 (limits +-pi/2, clamp +-pi), P=4096,
       I=500, B=8192

and the DH rows of SURVEY.md §8(f) row 4 (not BASELINE configs; bench.py
--config dh7*): the 7-joint KUKA iiwa 14 as a DH arm, 4096 reachable targets
(tool positions of seeded joint angles), P=1024, I=500, position-only fitness:
    dh7         joint-axis mask, D = 7 (FAST: the folded chain)
    dh7-nofold  joint-axis mask, D = 7, Euler kernels skipping locked angles
    dh7-locked  no mask: locked angles emulated by equal clamp bounds, D = 33

Particle seeds are global: swarm b, particle i uses curand_init(b*P + i), so
swarm 0 of config 3 is the reference's own solve and any sharding of the batch
reproduces the same per-swarm results.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from .scene import RESET_TARGETS, reference_scene, serial_chain
from .solver import MAIN_FITNESS, FitnessConfig, PSOConfig

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64_stream(seeds: np.ndarray, count: int) -> np.ndarray:
    """`count` successive splitmix64 outputs for each uint64 seed: [len(seeds), count]."""
    state = np.asarray(seeds, dtype=np.uint64).copy()
    out = np.empty((state.size, count), dtype=np.uint64)
    with np.errstate(over="ignore"):
        for j in range(count):
            state = state + np.uint64(0x9E3779B97F4A7C15)
            z = state.copy()
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            out[:, j] = z ^ (z >> np.uint64(31))
    return out


def unit_floats(u64: np.ndarray) -> np.ndarray:
    """Top 24 bits -> float in [0, 1)."""
    return ((u64 >> np.uint64(40)).astype(np.float64) / float(1 << 24))


def batch_targets(first_swarm: int, count: int) -> np.ndarray:
    """Config 3/4 targets for global swarms [first, first+count): [count, 3, 3] float32."""
    b = np.arange(first_swarm, first_swarm + count, dtype=np.uint64)
    u = unit_floats(splitmix64_stream(np.uint64(0x5EED0000) + b, 9)).reshape(count, 3, 3)
    return (RESET_TARGETS[None].astype(np.float64) + (u - 0.5) * 0.5).astype(np.float32)


def shell_targets(first_swarm: int, count: int, r_lo: float = 2.0, r_hi: float = 4.0) -> np.ndarray:
    """Config 5 tip targets uniformly in a spherical shell: [count, 1, 3] float32."""
    b = np.arange(first_swarm, first_swarm + count, dtype=np.uint64)
    u = unit_floats(splitmix64_stream(np.uint64(0x5EED5000) + b, 3))
    r = r_lo + (r_hi - r_lo) * u[:, 0]
    ct = 2.0 * u[:, 1] - 1.0
    st = np.sqrt(np.maximum(0.0, 1.0 - ct * ct))
    ph = 2.0 * np.pi * u[:, 2]
    p = np.stack([r * st * np.cos(ph), r * st * np.sin(ph), r * ct], axis=1)
    return p.astype(np.float32)[:, None, :]


@dataclass
class Workload:
    name: str
    chain: np.ndarray
    particles: int
    iterations: int
    swarms: int
    pso: PSOConfig
    fit: FitnessConfig
    limit_weight: float = 0.0
    soft_lo: Optional[np.ndarray] = None
    soft_hi: Optional[np.ndarray] = None
    description: str = ""
    extra: dict = field(default_factory=dict)
    axis_mask: Optional[np.ndarray] = None
    fold: bool = True

    @property
    def dof(self) -> int:
        if self.axis_mask is not None:
            return int(sum(bin(int(m) & 7).count("1") for m in self.axis_mask[1:]))
        return 3 * (self.chain.shape[0] - 1)

    def targets(self, first_swarm: int, count: int) -> np.ndarray:
        if self.name == "config5":
            return shell_targets(first_swarm, count)
        if self.name.startswith("dh7"):
            return dh7_targets(first_swarm, count)
        if self.name in ("config1", "config2"):
            return np.repeat(RESET_TARGETS[None], count, axis=0)
        return batch_targets(first_swarm, count)


def dh7_targets(first_swarm: int, count: int) -> np.ndarray:
    """Reachable iiwa tool positions: the DH product of joint angles U(-0.8, 0.8)
    x limits from splitmix64(0x5EED7000 + b): [count, 1, 3] float32."""
    from .dh import IIWA14, dh_forward

    b = np.arange(first_swarm, first_swarm + count, dtype=np.uint64)
    u = unit_floats(splitmix64_stream(np.uint64(0x5EED7000) + b, 7))
    th = (2.0 * u - 1.0) * 0.8 * IIWA14["limits"][None]
    p = np.array([dh_forward(t, IIWA14["d"], IIWA14["a"], IIWA14["alpha"]) for t in th])
    return p.astype(np.float32)[:, None, :]


def workload(n) -> Workload:
    pso = PSOConfig(0.5, 0.5, 1.25, 500)  # src/Main.cpp:130 coefficients
    if n in (1, 2, 3, 4):
        chain = reference_scene(reset=True).origin.to_cuda()
        P, I, B = {1: (256, 200, 1), 2: (1024, 500, 1), 3: (1024, 500, 4096), 4: (1024, 500, 65536)}[n]
        pso = PSOConfig(0.5, 0.5, 1.25, I)
        desc = {
            1: "reference scene, reset targets, 1 swarm (CPU plumbing)",
            2: "reference scene, reset targets, 1 swarm",
            3: "7-joint (21-DOF) reference scene, perturbed reset targets",
            4: "7-joint (21-DOF) reference scene, perturbed reset targets, sharded over the GPUs",
        }[n]
        return Workload(f"config{n}", chain, P, I, B, pso, MAIN_FITNESS, description=desc)
    if n == 5:
        origin = serial_chain(20, 0.25, rotation=(0.0, 0.3, 0.0))
        chain = origin.to_cuda()
        D = 60
        soft = np.full(D, np.pi / 2, dtype=np.float32)
        return Workload("config5", chain, 4096, 500, 8192, pso, MAIN_FITNESS, limit_weight=10.0, soft_lo=-soft,
                        soft_hi=soft,
                        description="20-joint serial chain (D=60), tip effector, targets in a radius-2..4 shell, "
                                    "soft joint-limit penalty")
    if isinstance(n, str) and n in ("dh7", "dh7-nofold", "dh7-locked"):
        from .dh import iiwa14

        arm = iiwa14()
        mask = None if n == "dh7-locked" else arm.axis_mask
        how = {"dh7": "joint-axis mask (D=7), folded chain",
               "dh7-nofold": "joint-axis mask (D=7), Euler kernels",
               "dh7-locked": "locked axes by equal clamp bounds (D=33)"}[n]
        return Workload(n, arm.origin.to_cuda(), 1024, 500, 4096, pso, FitnessConfig(0.0, 0.0, 0.1),
                        description=f"7-joint KUKA iiwa 14 DH arm as 11 nodes, {how}, reachable targets, "
                                    "position-only fitness",
                        axis_mask=mask, fold=n == "dh7")
    if isinstance(n, str) and n.isdigit():
        return workload(int(n))
    raise ValueError(f"no BASELINE config {n}")
