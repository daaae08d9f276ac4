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


FIXTURE_DIR = __import__("pathlib").Path(__file__).resolve().parent / "golden"
# SURVEY.md §8(c) tier-B tolerances per swarm: |df|/f, |dr|, effector positions through FK
TOLS = (("rel_fitness", 1e-3), ("residual_abs", 1e-3), ("effector_pos_abs", 1e-2))


def load_fixture(cfg) -> dict:
    """tests/golden/tierb_config{cfg}.npz, or tierb_collide.npz for cfg "collide" (config 3 with
    the reference's collider boxes 0 and 3; tests/golden/make_tierb.py): the oracle's answers
    (ref: -ffp-contract=off, the parity checker) and the same solves with FMA contraction (fma)."""
    name = "tierb_collide.npz" if cfg == "collide" else f"tierb_config{cfg}.npz"
    with np.load(FIXTURE_DIR / name) as z:
        return {k: z[k] for k in z.files}


def envelope(chain, fx: dict):
    """Per-swarm tier-B distances of the FMA-contracted oracle from the parity oracle."""
    return tier_b_distances(chain, fx["fma_angles"], fx["fma_fitness"], fx["fma_residual"], fx["ref_angles"],
                            fx["ref_fitness"], fx["ref_residual"])


# The paired fitness comparison is strict: only exactly equal fitness values are ties.
# Round 5 counted relative differences within 1e-5 as ties, to absorb a measured bias of the
# transcendental unit's sin/cos (amplitude -3.2e-8, compounding over config 5's 60 plane
# rotations to a median +1.4e-6 of the final fitness: strict count 83 worse / 44 better,
# p = 3e-4).  Round 6 removes the bias at its source -- the FAST kernels on the
# transcendental unit scale each link length by its expected shrink (kHwTrigAmplitudeBias,
# ikpso_kernels.h) -- so the strict test is the asserted one.  The count with a 1e-5 tie
# window is still reported (tie_window).
SIGN_TIE = 0.0
SIGN_TIE_REPORTED = 1e-5
# Absolute floor beside the Fisher test: the GPU's share of swarms within each tolerance
# may not fall more than this below the envelope's, whatever the test's power.
SHARE_FLOOR = 0.05


def stat_tests(dist, env, fit, ref_fit, tie: float = SIGN_TIE):
    """The FAST-parity decision, stated as tests (alpha = 0.01):
      * per tolerance of TOLS: one-sided Fisher exact test of H0 "the GPU's share of swarms
        within the tolerance is at least the envelope's" (two valid fp32 evaluations of the
        same solves) against "it is lower" -- fails when p < 0.01; and an absolute floor: the
        share may not be more than SHARE_FLOOR below the envelope's;
      * a paired sign test of the per-swarm gbest fitness: H0 "the GPU's answer is as likely
        better than the oracle's as worse" against "worse", exactly equal values counted as
        ties (`tie`: relative differences within it) -- fails when p < 0.01.  The same count
        with the 1e-5 window round 5 used is reported (tie_window), not asserted.
    Returns a report dict with the shares, p-values and verdicts."""
    from scipy.stats import binomtest, fisher_exact

    out = {}
    n = len(fit)
    for (name, tol), d, e in zip(TOLS, dist, env):
        kg, ke = int(np.sum(d <= tol)), int(np.sum(e <= tol))
        p = float(fisher_exact([[kg, n - kg], [ke, n - ke]], alternative="less")[1])
        floor_ok = kg / n >= ke / n - SHARE_FLOOR
        out[name] = {"tol": tol, "gpu_within": kg, "envelope_within": ke, "swarms": n, "fisher_p_lower": p,
                     "share_floor": SHARE_FLOOR, "pass": p >= 0.01 and floor_ok}

    def sign(t):
        rel = (np.asarray(fit, np.float64) - ref_fit) / np.asarray(ref_fit, np.float64)
        worse, better = int(np.sum(rel > t)), int(np.sum(rel < -t))
        p = float(binomtest(worse, worse + better, 0.5, alternative="greater").pvalue) if worse + better else 1.0
        return worse, better, p, float(np.median(rel))

    worse, better, p, med = sign(tie)
    tw, tb, tp, _ = sign(SIGN_TIE_REPORTED)
    out["fitness_sign"] = {"tie": tie, "worse": worse, "better": better, "ties": n - worse - better,
                           "sign_p_worse": p, "pass": p >= 0.01, "median_rel_diff": med,
                           "tie_window": {"tie": SIGN_TIE_REPORTED, "worse": tw, "better": tb, "sign_p_worse": tp},
                           "mean_fitness": float(np.mean(fit)), "oracle_mean_fitness": float(np.mean(ref_fit))}
    out["pass"] = all(v["pass"] for v in out.values() if isinstance(v, dict))
    return out
