"""BASELINE config 5 at its own configuration, against the CPU oracle.

The benchmarked config-5 kernel is k_swarm_coop<TopoSerialTip<20>>: a swarm of
4096 particles of the 20-joint chain (D = 60) over G = 16 co-resident 256-lane
chunks (two chunks of different swarms per CU), exchanging chunk minima through
L2 every iteration, with the soft joint-limit penalty.  Reference semantics: calculatePSO,
src/kernel.cu:279-327 (init, then I x update / evaluate / first-minimum argmin /
strict global-best improvement); SURVEY.md §8(c) tiers A and B.

  * REFERENCE arithmetic, 2 swarms x 4096 x I = 20: bit-exact angles, fitness
    and generator states (the draw count is integer work);
  * FAST arithmetic, tier B, 128 swarms x 4096 x I = 500 (chaotic regime), per
    swarm against SURVEY.md §8(c)'s tolerances (|df|/f <= 1e-3, residual within
    1e-3, tip position of the answer within 1e-2 through FK), decided by stated
    tests against the oracle's own FMA on/off envelope on the same swarms (the
    per-swarm bounds are the dynamics', not the kernel's: two valid fp32
    evaluations one rounding apart do not meet them on every swarm): one-sided
    Fisher exact tests of the shares, a sign test of the fitness (tests/tierb.py,
    alpha = 0.01); no swarm further than twice the envelope's worst swarm on each
    distance; median |df|/f <= 1e-4, mean fitness within 0.5 %, generator states
    bit-exact;
  * the cooperative solve's streaming fallback (and an explicit streaming solve)
    evaluate the tip from the tip back like the cooperative kernel, so FAST
    results agree across the families (I <= 10: |dtheta| <= 1e-3, |df|/f <= 1e-4).
"""
import numpy as np
import pytest

import ikpso
from tierb import envelope, load_fixture, stat_tests, tier_b_distances, tier_b_report

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
    """128 swarms x 4096 particles x 500 iterations (the benchmarked kernel, FAST)
    against the oracle's answers in tests/golden/tierb_config5.npz, with the
    oracle's FMA on/off envelope on the same swarms and the stated tests of
    tests/tierb.py (stat_tests, alpha = 0.01)."""
    wl = ikpso.workload(5)
    fx = load_fixture(5)
    B, I, P, D = int(fx["swarms"]), wl.iterations, wl.particles, wl.dof
    tg = wl.targets(0, B)
    wl, s = config5_solver("fast", I)
    assert s.kernel == "swarm_coop<serial_tip20>", s.kernel
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    assert s.kernel == "swarm_coop<serial_tip20>", s.kernel  # the throughput plan (not the latency name)
    states = s.generator_states(0, B)
    s.close()
    assert np.array_equal(states[:, :6], words(oracle.skipahead(oracle.init_generators(B * P, 0), D + 3 * D * I)))
    assert np.isfinite(fit).all() and np.isfinite(ang).all()
    rang, rfit, rres = fx["ref_angles"], fx["ref_fitness"], fx["ref_residual"]
    env = envelope(wl.chain, fx)
    dist = tier_b_distances(wl.chain, ang, fit, res, rang, rfit, rres)
    rep = tier_b_report(*dist)
    tests = stat_tests(dist, env, fit, rfit)
    rep.update(mean_fitness=float(fit.mean()), oracle_mean_fitness=float(rfit.mean()), envelope=tier_b_report(*env),
               tests=tests)
    report("tier_b_config5", rep)
    assert tests["pass"], tests
    rel, dres, dpos = dist
    assert np.median(rel) <= 1e-4, np.median(rel)
    # gross-error ceilings: twice the envelope's worst swarm on the same batch
    for d, e in zip(dist, env):
        assert d.max() <= 2 * e.max(), (d.max(), e.max())
    assert abs(fit.mean() - rfit.mean()) / rfit.mean() < 5e-3
    assert abs(res.mean() - rres.mean()) < 1e-3 + 0.01 * rres.mean()
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
