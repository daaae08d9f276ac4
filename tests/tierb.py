"""Tier-B distances shared by the GPU parity tests; test
infrastructure (the oracle's FK is the checker)."""
import numpy as np

import ikpso
import oracle


def tier_b_distances(chain, ang, fit, res, oang, ofit, ores):
    """Per-swarm tier-B distances: |df|/f of the gbest fitness,
    |dr| of the residual, and the largest effector-position difference of the two
    answers through the oracle's FK (effector targets do not enter the FK)."""
    eff = np.flatnonzero(chain["node_type"] == ikpso.NODE_EFFECTOR)
    rel = np.abs(fit - ofit) / ofit
    dres = np.abs(res - ores)
    dpos = np.array([np.max(np.abs(oracle.node_positions(chain, ang[b])[eff - 1] - oracle.node_positions(chain, oang[b])[eff - 1]))
                     for b in range(len(fit))])
    return rel, dres, dpos


def tier_b_report(rel, dres, dpos):
    q = lambda x: {"median": float(np.median(x)), "p90": float(np.percentile(x, 90)), "max": float(x.max())}
    return {"swarms": int(len(rel)), "rel_fitness": q(rel), "residual_abs": q(dres), "effector_pos_abs": q(dpos),
            "frac_rel_le_1e-3": float(np.mean(rel <= 1e-3)), "frac_res_le_1e-3": float(np.mean(dres <= 1e-3)),
            "frac_pos_le_1e-2": float(np.mean(dpos <= 1e-2))}
