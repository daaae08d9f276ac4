"""BASELINE config 5 at its own configuration, against the CPU oracle.

The benchmarked config-5 kernel is k_swarm_coop<TopoSerialTip<20>>: a swarm of
4096 particles of the 20-joint chain (D = 60) over G = 16 co-resident 256-lane
chunks (two chunks of different swarms per CU), exchanging chunk minima through
L2 every iteration, with the soft joint-limit penalty.  Reference semantics: calculatePSO,
src/kernel.cu:279-327 (init, then I x update / evaluate / first-minimum argmin /
strict global-best improvement); SURVEY.md §8(c) tiers A and B.

  * REFERENCE arithmetic, 2 swarms x 4096 x I = 20: bit-exact angles, fitness
    and generator states (the draw count is integer work);
  * FAST arithmetic, tier B, 32 swarms x 4096 x I = 500 (chaotic regime), per
    swarm against SURVEY.md §8(c)'s tolerances (|df|/f <= 1e-3, residual within
    1e-3, tip position of the answer within 1e-2 through FK): >= 80 % of swarms
    within each, every swarm within |df|/f <= 1e-2, |dr| <= 0.1, tip <= 0.2;
    median |df|/f <= 1e-4, mean fitness within 0.5 %, generator states bit-exact.
    The per-swarm bounds are the dynamics', not the kernel's: the oracle itself,
    built with and without FMA contraction (two valid fp32 evaluations one
    rounding apart), meets the tolerances on 94 / 91 / 94 % of these swarms,
    worst 2.8e-3 / 1.3e-2 / 1.3e-2 (tools/tier_b_envelope.py,
    profiles/r04/tier_b_envelope.json);
  * the cooperative solve's streaming fallback (and an explicit streaming solve)
    evaluate the tip from the tip back like the cooperative kernel, so FAST
    results agree across the families (I <= 10: |dtheta| <= 1e-3, |df|/f <= 1e-4).
"""
import numpy as np
import pytest

import ikpso
from tierb import tier_b_distances, tier_b_report

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def words(states):
    return states.view(np.int32).reshape(-1, 12)[:, :6]


def config5_solver(arith, I, kernel="auto"):
    wl = ikpso.workload(5)
    s = ikpso.BatchSolver(wl.chain, wl.particles, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith=arith,
                          limit_weight=wl.limit_weight, soft_lo=wl.soft_lo, soft_hi=wl.soft_hi, kernel=kernel)
    return wl, s


def oracle_batch(oracle, wl, B, I, threads=0):
    try:
        lib = oracle.load_native()  # -O3 -march=native, same source and results (-ffp-contract=off)
    except Exception:
        lib = None
    tg = wl.targets(0, B)
    ostate = oracle.init_generators(B * wl.particles, 0)
    kw = {"lib": lib} if lib is not None else {}
    oang, ofit, ores = oracle.solve_batch(wl.chain, tg, None, wl.particles, I, ostate, limit_weight=wl.limit_weight,
                                          soft_lo=wl.soft_lo, soft_hi=wl.soft_hi, threads=threads, **kw)
    return tg, oang, ofit, ores, ostate


def test_config5_reference_bitexact_g16(oracle, device):
    """2 swarms x 4096 particles x 20 iterations through k_swarm_coop with G = 16."""
    B, I = 2, 20
    wl, s = config5_solver("reference", I)
    assert s.kernel == "swarm_coop<serial_tip20>", s.kernel
    assert wl.particles == 4096
    s.seed(B)
    tg, oang, ofit, ores, ostate = oracle_batch(oracle, wl, B, I)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    assert s.kernel == "swarm_coop<serial_tip20>", s.kernel  # the throughput plan (not the latency name)
    states = s.generator_states(0, B)
    s.close()
    assert np.array_equal(states[:, :6], words(ostate))  # D + 3*D*I draws per particle
    assert np.array_equal(ang, oang)
    assert np.array_equal(fit, ofit)
    assert np.max(np.abs(res - ores)) <= 1e-5


def test_config5_fast_tier_b_own_size(oracle, device, report):
    """32 swarms x 4096 particles x 500 iterations (the benchmarked kernel, FAST)."""
    B, I = 32, 500
    wl, s = config5_solver("fast", I)
    assert s.kernel == "swarm_coop<serial_tip20>", s.kernel
    s.seed(B)
    tg, oang, ofit, ores, ostate = oracle_batch(oracle, wl, B, I)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    assert s.kernel == "swarm_coop<serial_tip20>", s.kernel  # the throughput plan (not the latency name)
    states = s.generator_states(0, B)
    s.close()
    assert np.array_equal(states[:, :6], words(ostate))
    assert np.isfinite(fit).all() and np.isfinite(ang).all()
    rel = np.abs(fit - ofit) / ofit
    frac = float(np.mean(rel <= 1e-3))
    print(f"tier B config 5: {frac:.3f} of {B} swarms within 1e-3; median |df|/f {np.median(rel):.2e}, "
          f"max {rel.max():.2e}; mean fitness {fit.mean():.6f} vs {ofit.mean():.6f}; "
          f"mean residual {res.mean():.5f} vs {ores.mean():.5f}")
    rel, dres, dpos = tier_b_distances(wl.chain, ang, fit, res, oang, ofit, ores)
    rep = tier_b_report(rel, dres, dpos)
    rep.update(mean_fitness=float(fit.mean()), oracle_mean_fitness=float(ofit.mean()))
    report("tier_b_config5", rep)
    assert frac >= 0.8, (frac, np.sort(rel)[-6:])
    assert rep["frac_res_le_1e-3"] >= 0.8 and rep["frac_pos_le_1e-2"] >= 0.8, rep
    assert rel.max() <= 1e-2 and np.median(rel) <= 1e-4, (np.median(rel), rel.max())
    assert dres.max() <= 0.1 and dpos.max() <= 0.2, rep  # gross-error ceilings (measured 0.013 / 0.023)
    assert abs(fit.mean() - ofit.mean()) / ofit.mean() < 5e-3
    assert abs(res.mean() - ores.mean()) < 1e-3 + 0.01 * ores.mean()
    # the reported fitness is the fitness of the reported angles (penalty included)
    eff = np.flatnonzero(wl.chain["node_type"] == ikpso.NODE_EFFECTOR)
    for b in range(B):
        ch = wl.chain.copy()
        ch["target_position"][eff] = tg[b]
        f = oracle.fitness(ch, ang[b], limit_weight=wl.limit_weight, soft_lo=wl.soft_lo, soft_hi=wl.soft_hi)
        assert abs(float(f) - float(fit[b])) <= 1e-5 * abs(float(f)) + 1e-6, (b, f, fit[b])


@pytest.mark.parametrize("I", [5, 10])
def test_config5_fast_families_agree(device, monkeypatch, I):
    """FAST: the cooperative kernel, its forced streaming fallback and an explicit
    streaming solve all evaluate the tip from the tip back (one rounding form), so
    they agree to the FAST tolerance (the backend fuses multiply-adds per kernel);
    generator states are identical."""
    B = 4
    out = {}
    for name, kernel, spin in (("coop", "coop", None), ("fallback", "coop", "0"), ("streaming", "streaming", None)):
        if spin is None:
            monkeypatch.delenv("IKPSO_COOP_SPIN_LIMIT", raising=False)
        else:
            monkeypatch.setenv("IKPSO_COOP_SPIN_LIMIT", spin)
        wl, s = config5_solver("fast", I, kernel=kernel)
        s.seed(B)
        r = [t.cpu().numpy() for t in s.solve(dev(wl.targets(0, B)), iterations=I)]
        if name == "fallback":
            assert s.fallbacks == 1
        out[name] = r + [s.generator_states(0, B)]
        s.close()
    ca, cf, cr, cs = out["coop"]
    for name in ("fallback", "streaming"):
        a, f, r, st = out[name]
        assert np.array_equal(st, cs), name
        assert np.max(np.abs(a - ca)) < 1e-3, (name, np.max(np.abs(a - ca)))
        assert np.max(np.abs(f - cf) / cf) < 1e-4, (name, np.max(np.abs(f - cf) / cf))
