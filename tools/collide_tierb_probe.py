#!/usr/bin/env python3
"""Experiment (GPU): where does a FAST collider build's tier-B bias come from?  The stated
tests of tests/tierb.py on
  far    config 3's fixture (tierb_config3.npz) solved by the collider build with every box out
         of reach (IKPSO_KEEP_FAR_COLLIDERS=1: the kernel, its sin/cos and pinned FK, no contact);
  near   the collide leg's fixture (tierb_collide.npz: boxes 0 and 3);
each with the unmasked collider build (the transcendental unit's sin/cos) and with an all-free
axis mask (the masked collider build: the polynomial sin/cos, same pinned FK).  Test
infrastructure (imports tests/tierb.py and the oracle)."""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "inverse-kinematics-pso-research_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import torch  # noqa: E402

import ikpso  # noqa: E402
from tierb import envelope, load_fixture, stat_tests, tier_b_distances  # noqa: E402


def run(name, fxname, boxes, mask):
    wl = ikpso.workload(3)
    fx = load_fixture(fxname)
    B = int(fx["swarms"])
    s = ikpso.BatchSolver(wl.chain, wl.particles, pso=wl.pso, colliders=boxes, axis_mask=mask)
    s.seed(B)
    tg = torch.from_numpy(wl.targets(0, B)).cuda()
    ang, fit, res = (t.cpu().numpy() for t in s.solve(tg, iterations=wl.iterations))
    out = {"case": name, "kernel": s.kernel, "colliders_tested": s.collider_count}
    s.close()
    t = stat_tests(tier_b_distances(wl.chain, ang, fit, res, fx["ref_angles"], fx["ref_fitness"], fx["ref_residual"]),
                   envelope(wl.chain, fx), fit, fx["ref_fitness"])
    sg = t["fitness_sign"]
    out.update(passed=t["pass"], worse=sg["worse"], better=sg["better"], p=round(sg["sign_p_worse"], 4),
               median=sg["median_rel_diff"], mean=sg["mean_fitness"], oracle_mean=sg["oracle_mean_fitness"])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    os.environ["IKPSO_KEEP_FAR_COLLIDERS"] = "1"
    far = ikpso.init_colliders(4)
    far["pos"] += 1000.0
    near = ikpso.init_colliders(4)[[0, 3]]
    allfree = np.array([0] + [7] * 7, np.uint8)
    for mask, trig in ((None, "hw"), (allfree, "poly")):
        run(f"far_{trig}", 3, far, mask)
        run(f"near_{trig}", "collide", near, mask)
