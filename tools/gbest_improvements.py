#!/usr/bin/env python3
"""How often a single config-2 solve's global best improves (CPU oracle, no GPU):
the solve of every iteration count 0..500 from the same seeds shares the
trajectory's prefix, so iteration i improved iff gbest(i) < gbest(i-1).
Prices a speculative exchange: an iteration computed with the
previous global best is kept unless the exchange it overlapped improved it."""
import sys
from multiprocessing import Pool
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "inverse-kinematics-pso-research_amd"))
sys.path.insert(0, str(ROOT))
import ikpso  # noqa: E402
from oracle import oracle  # noqa: E402

WL = ikpso.workload(2)


def run(args):
    t, i = args
    st = oracle.init_generators(WL.particles, t * WL.particles)
    _, fit, _ = oracle.solve_batch(WL.chain, WL.targets(t, 1), None, WL.particles, i, st, threads=1)
    return t, i, float(fit[0])


if __name__ == "__main__":
    targets = range(int(sys.argv[1]) if len(sys.argv) > 1 else 2)
    jobs = [(t, i) for t in targets for i in range(WL.iterations + 1)]
    with Pool(8) as p:
        out = p.map(run, jobs, chunksize=4)
    for t in targets:
        f = np.array([x[2] for x in out if x[0] == t])
        imp = f[1:] < f[:-1]
        print(f"target {t}: {imp.sum()} of {len(imp)} iterations improve the global best "
              f"(iterations 1-50: {imp[:50].sum()}, 51-100: {imp[50:100].sum()}, 101-500: {imp[100:].sum()}); "
              f"final fitness {f[-1]:.6f}")
