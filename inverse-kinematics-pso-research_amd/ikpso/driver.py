"""Per-frame warm-start driver: the reference visualiser's solve loop without
the window.

Reference frame loop (src/Main.cpp:163-250, src/ = InverseKinematicsResearch/
InverseKinematicsResearch/):
    if recording: framesCounter++; write the diagnostics logs; dist =
        checkDistance(effectors); if dist <= epsDist: resetArm(), log
        framesCounter, framesCounter = 0                     (:171-215)
    nodeArm->ToCUDA(chain); nodeArm->FillPositions(positions) (:222-223)
    calculatePSO(...); nodeArm->FromCoords(result)           (:225-227)
The generator states persist across frames and test cases (initGenerators is
called once, :145).  A recorded "frames to converge" therefore counts the
solves needed plus the frame that observes convergence.

Diagnostics logs (src/Main.cpp:147-154,178-202,300-328): four append-mode
text files in the working directory, values written with C++ ostream's
default formatting (%g, 6 significant digits), ';'-terminated per value.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .scene import Scene, reference_scene
from .solver import MAIN_FITNESS, MAIN_PSO, FitnessConfig, PSOConfig, calculate_pso, init_generators

LOG_FILES = ("IK-diagnostics-positions.txt", "IK-diagnostics-degrees.txt", "IK-diagnostics-frames.txt",
             "IK-diagnostics-distance.txt")


def _g(x: float) -> str:
    return "%g" % float(np.float32(x))


@dataclass
class DiagnosticsLog:
    """The four IK-diagnostics-*.txt streams (append mode, like openStream, src/Main.cpp:300-304)."""

    directory: str
    _files: list = field(default_factory=list)

    def __post_init__(self):
        os.makedirs(self.directory, exist_ok=True)
        self._files = [open(os.path.join(self.directory, n), "a") for n in LOG_FILES]

    def frame(self, positions: np.ndarray, degrees: np.ndarray, distance: float) -> None:
        pos, deg, _, dist = self._files
        deg.write("".join(_g(v) + ";" for v in degrees) + "\n")
        pos.write("".join(_g(v) + ";" for v in positions) + "\n")
        dist.write(_g(distance) + "\n")

    def converged(self, frames: int) -> None:
        self._files[2].write(f"{frames}\n")

    def close(self) -> None:
        for f in self._files:
            f.close()


class FrameDriver:
    """Runs test cases the way the visualiser records them (R pressed: reset
    the arm, count frames until the effector distance sum <= eps)."""

    def __init__(self, particles: int = 16384, pso: PSOConfig = MAIN_PSO, fit: FitnessConfig = MAIN_FITNESS,
                 scene: Optional[Scene] = None, log_dir: Optional[str] = None, device="cuda", colliders=None):
        import torch

        self.torch = torch
        self.N = int(particles)
        self.pso, self.fit = pso, fit
        self.scene = scene or reference_scene(reset=True)
        self.D = self.scene.origin.to_coords().size
        # caller-owned buffers, as src/Main.cpp:137-141
        self.particles = torch.zeros((3, self.D, self.N), dtype=torch.float32, device=device)
        self.bests = torch.zeros(self.N, dtype=torch.float32, device=device)
        self.randoms = torch.zeros((self.N, 12), dtype=torch.int32, device=device)
        self.result = np.zeros(self.D, dtype=np.float32)
        st = init_generators(self.randoms, self.N)
        if st != 0:
            raise RuntimeError(f"initGenerators failed ({st})")
        self.log = DiagnosticsLog(log_dir) if log_dir else None
        # obj_t colliders (initColliders, src/Main.cpp:140-144); none by default, as src/Main.cpp:18
        self.colliders = colliders

    def solve_frame(self) -> None:
        chain = self.scene.origin.to_cuda()
        positions = self.scene.origin.fill_positions()
        nc = 0 if self.colliders is None else len(self.colliders)
        st = calculate_pso(self.particles, positions, self.bests, self.randoms, self.N, chain, self.pso, self.fit,
                           self.result, self.colliders if nc else None, nc)
        if st != 0:  # the frame loop breaks on a failed solve (src/Main.cpp:226)
            raise RuntimeError(f"calculatePSO failed ({st})")
        self.scene.origin.from_coords(self.result)

    def _positions(self) -> np.ndarray:
        return np.concatenate([n.world_position() for n in list(self.scene.origin.dfs())[1:]])

    def run_case(self, eps: float = 0.025, max_frames: int = 2000) -> int:
        """One recorded test case; returns the logged frame count (-1 if max_frames hit)."""
        self.scene.reset_arm()
        frames = 0
        while frames < max_frames:
            frames += 1
            dist = self.scene.check_distance()
            if self.log:
                self.log.frame(self._positions(), self.result, dist)
            if dist <= eps:
                self.scene.reset_arm()
                if self.log:
                    self.log.converged(frames)
                return frames
            self.solve_frame()
        return -1

    def run_cases(self, n: int, eps: float = 0.025, max_frames: int = 2000) -> List[int]:
        return [self.run_case(eps, max_frames) for _ in range(n)]

    def close(self) -> None:
        if self.log:
            self.log.close()
