#!/usr/bin/env python3
"""Tier-B envelope: how far two VALID fp32 evaluations of the same PSO solve end
apart after 500 chaotic iterations -- the CPU oracle built without FMA
contraction (the parity oracle) and with it (-mfma -ffp-contract=fast), same
seeds, same targets (SURVEY.md §8(c) "Measured divergence").

The FAST GPU kernels differ from the oracle by roundings of that kind, so the
per-swarm tier-B bounds in tests/test_gpu_parity.py (config 3) and
tests/test_gpu_config5.py (config 5) are set from this distribution: the share of
swarms within SURVEY's per-swarm tolerances (|df|/f <= 1e-3, residual within 1e-3,
effector positions within 1e-2), and a ceiling above the envelope's worst swarm.
Writes profiles/r04/tier_b_envelope.json.  Test infrastructure (imports oracle/).
"""
from __future__ import annotations

import ctypes
import json
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "inverse-kinematics-pso-research_amd")]

import ikpso  # noqa: E402
import oracle  # noqa: E402


def fma_oracle():
    out = Path(tempfile.mkdtemp()) / "libikpso_oracle_fma.so"
    src = [str(ROOT / "oracle" / "ikpso_oracle.c"), str(ROOT / "oracle" / "ikpso_gjk.c")]
    subprocess.run(["gcc", "-O2", "-std=c11", "-march=native", "-mfma", "-ffp-contract=fast", "-fopenmp", "-fPIC",
                    "-shared", *src, "-o", str(out), "-lm"], check=True)
    return oracle._bind(ctypes.CDLL(str(out)))


def tier_b_metrics(chain, a1, f1, r1, a2, f2, r2, limit_kw=None):
    """Per-swarm distances between two solves of the same batch."""
    eff = np.flatnonzero(chain["node_type"] == ikpso.NODE_EFFECTOR)
    rel = np.abs(f1 - f2) / f1
    dres = np.abs(r1 - r2)
    dpos = np.array([np.max(np.abs(oracle.node_positions(chain, a1[b])[eff - 1] -
                                   oracle.node_positions(chain, a2[b])[eff - 1])) for b in range(len(f1))])
    return rel, dres, dpos


def summary(rel, dres, dpos):
    q = lambda x: {"median": float(np.median(x)), "p90": float(np.percentile(x, 90)), "max": float(x.max())}
    return {"swarms": int(len(rel)), "rel_fitness": q(rel), "residual_abs": q(dres), "effector_pos_abs": q(dpos),
            "frac_rel_le_1e-3": float(np.mean(rel <= 1e-3)), "frac_res_le_1e-3": float(np.mean(dres <= 1e-3)),
            "frac_pos_le_1e-2": float(np.mean(dpos <= 1e-2))}


def main():
    fma = fma_oracle()
    out = {"note": __doc__.strip().splitlines()[0] + " -- oracle (-ffp-contract=off) vs oracle (FMA contraction)"}
    for cfg, B in ((3, 64), (5, 32)):
        wl = ikpso.workload(cfg)
        P, I = wl.particles, wl.iterations
        tg = wl.targets(0, B)
        kw = dict(limit_weight=wl.limit_weight, soft_lo=wl.soft_lo, soft_hi=wl.soft_hi)
        a1, f1, r1 = oracle.solve_batch(wl.chain, tg, None, P, I, oracle.init_generators(B * P, 0), threads=0, **kw)
        a2, f2, r2 = oracle.solve_batch(wl.chain, tg, None, P, I, oracle.init_generators(B * P, 0), threads=0,
                                        lib=fma, **kw)
        s = summary(*tier_b_metrics(wl.chain, a1, f1, r1, a2, f2, r2))
        s["workload"] = f"config {cfg}: {B} swarms x {P} particles x {I} iterations (the GPU tier-B batch)"
        out[f"config{cfg}"] = s
        print(cfg, json.dumps(s))
    dst = ROOT / "profiles" / "r04" / "tier_b_envelope.json"
    dst.parent.mkdir(parents=True, exist_ok=True)
    dst.write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
