#!/usr/bin/env python3
"""Cost of the collider term (src/kernel.cu:104-136): config 3's
batch solved with no colliders (the plain kernel), with the reference's four
initColliders boxes moved 1000 units away (the collider kernel, every box pair
rejected by the bounding-sphere test: its FK-side cost without GJK), with the
boxes of src/Main.cpp:537-559 in place, and with boxes 0 and 3 only (which
leave the reset pose clear).  usage: collide_probe.py [SWARMS] [ITERS] [ARITH]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "inverse-kinematics-pso-research_amd"))
import numpy as np
import torch

import ikpso

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
I = int(sys.argv[2]) if len(sys.argv) > 2 else 500
arith = sys.argv[3] if len(sys.argv) > 3 else "fast"
wl = ikpso.workload(3)
P = wl.particles
tg = torch.from_numpy(np.ascontiguousarray(wl.targets(0, B))).cuda()
boxes = ikpso.init_colliders(4)
far = boxes.copy()
far["pos"] += 1000.0
cases = {"none": None, "far4": far, "init4": boxes, "init03": boxes[[0, 3]]}
for name, c in cases.items():
    s = ikpso.BatchSolver(wl.chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith=arith, colliders=c)
    s.seed(B)
    s.solve(tg, iterations=I)
    torch.cuda.synchronize()
    ms = []
    for _ in range(3):
        s.seed(B)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ang, fit, res = s.solve(tg, iterations=I)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    f = fit.cpu().numpy()
    print(f"{name:7s} {s.kernel:40s} {np.median(ms):9.3f} ms  {B * P * I / np.median(ms) / 1e6:.3e} upd/s  "
          f"mean fitness {f[f < 1e30].mean() if (f < 1e30).any() else float('nan'):.5f}  "
          f"FLT_MAX answers {int((f > 1e30).sum())}", flush=True)
    s.close()
