"""CPU oracle pinned against the reference's own recorded data and rocRAND.

The reference has no tests; its recorded diagnostics (Documentation/results.xlsx,
written by src/Main.cpp:147-215) are the known-answer data used here.
"""
import json

import numpy as np
import pytest

import ikpso


def test_xorwow_step_matches_rocrand(oracle, golden):
    """The XORWOW recurrence (curand(), restated) equals rocRAND's xorwow_engine::next()."""
    g = json.load(open(golden / "xorwow_rocrand.json"))
    for seed, state, draws in zip(g["seeds"], g["states"], g["draws"]):
        st = oracle.init_generators(1, seed)
        assert int(st["d"][0]) == state[0] and list(map(int, st["v"][0])) == state[1:], seed
        got = oracle.raw_stream(st, len(draws))
        assert got.tolist() == draws, seed


def test_curand_uniform_mapping(oracle):
    st = oracle.init_generators(1, 7)
    raw = oracle.raw_stream(st.copy(), 1000).astype(np.float32)
    u = oracle.uniform_stream(st, 1000)
    want = (raw * np.float32(2.3283064e-10) + np.float32(2.3283064e-10 / 2)).astype(np.float32)
    assert np.array_equal(u, want)
    assert np.all(u > 0) and np.all(u <= 1)


def test_seed_layout_is_global(oracle):
    """Generator i of a block seeded at base b equals generator b+i of base 0."""
    a = oracle.init_generators(64, 0)
    b = oracle.init_generators(16, 40)
    assert a[40:56].tobytes() == b.tobytes()


def test_fk_matches_recorded_positions(oracle, fk_kat):
    """Oracle FK (reference 4x4 order, fp32) vs 1583 recorded (angles -> positions) rows."""
    chain = ikpso.reference_scene().origin.to_cuda()
    deg, pos = fk_kat["degrees"], fk_kat["positions"]
    assert deg.shape == (1583, 21)
    errs = np.array([np.max(np.abs(oracle.node_positions(chain, a).ravel() - p)) for a, p in zip(deg, pos)])
    # positions were logged with 6 significant digits from unrounded angles
    assert errs.max() < 1e-4, errs.max()
    assert np.median(errs) < 3e-5  # angles themselves were logged with 6 digits


def test_residual_matches_recorded_distance(oracle, distance_kat):
    """checkDistance restated (sum of effector distances) vs the DISTANCE_1 log."""
    chain = ikpso.reference_scene(reset=True).origin.to_cuda()
    got = np.array([oracle.residual(chain, a) for a in distance_kat["degrees"]])
    assert np.max(np.abs(got - distance_kat["distance"])) < 2e-4


def test_fitness_terms(oracle):
    """Fitness at the rest pose is the effector term only; angle term is (aw/J)*|dtheta|^2."""
    scene = ikpso.reference_scene()
    chain = scene.origin.to_cuda()
    rest = scene.origin.to_coords()
    pos = oracle.node_positions(chain, rest)
    eff = sum(float(np.sum((pos[k - 1] - chain[k]["target_position"]) ** 2)) for k in (5, 6, 7))
    f0 = float(oracle.fitness(chain, rest, 3.0, 0.0))
    assert abs(f0 - eff) < 1e-5 * max(1.0, eff)
    bumped = rest.copy()
    bumped[0] += 0.5
    pos1 = oracle.node_positions(chain, bumped)
    eff1 = sum(float(np.sum((pos1[k - 1] - chain[k]["target_position"]) ** 2)) for k in (5, 6, 7))
    assert abs(float(oracle.fitness(chain, bumped, 3.0, 0.0)) - (eff1 + 3.0 / 7 * 0.25)) < 1e-5


def test_calculate_pso_invariants(oracle):
    """Draw count, pbest monotonicity, result = pbest of the first minimum."""
    scene = ikpso.reference_scene()
    chain = scene.origin.to_cuda()
    P, I, D = 64, 10, 21
    rng = oracle.init_generators(P, 0)
    rng0 = rng.copy()
    res, parts, bests = oracle.calculate_pso(chain, P, rng, iterations=I)
    # every particle consumed exactly D + 3*D*I uniforms
    for i in (0, 17, 63):
        s = rng0[i:i + 1].copy()
        oracle.raw_stream(s, D + 3 * D * I)
        assert s.tobytes() == rng[i:i + 1].tobytes()
    g = int(np.argmin(bests))
    assert np.array_equal(res, parts[2, :, g])
    fit_pb = np.array([oracle.fitness(chain, parts[2, :, i]) for i in range(P)], dtype=np.float32)
    assert np.array_equal(fit_pb, bests)
    # clamp to [0, 2pi]
    assert parts[0].min() >= 0.0 and parts[0].max() <= ikpso.scene.TWO_PI_F
    # pbest never worse than the start pose
    f_rest = oracle.fitness(chain, scene.origin.to_coords())
    assert np.all(bests <= f_rest)


def test_batch_equals_single_solves(oracle):
    """orc_solve_batch(b) == calculate_pso on swarm b's own chain and seeds."""
    wl = ikpso.workload(3)
    B, P, I = 3, 64, 5
    tg = wl.targets(0, B)
    rng = oracle.init_generators(B * P, 0)
    ang, fit, res = oracle.solve_batch(wl.chain, tg, None, P, I, rng.copy(), threads=2)
    for b in range(B):
        ch = wl.chain.copy()
        ch["target_position"][5:8] = tg[b]
        r1, _, bests = oracle.calculate_pso(ch, P, rng[b * P:(b + 1) * P].copy(), iterations=I)
        assert np.array_equal(r1, ang[b])
        assert fit[b] == bests.min()
        assert res[b] == oracle.residual(ch, r1)


def test_config1_converges(oracle):
    """Config 1 (CPU plumbing): 256 particles x 200 iterations improve on the start pose."""
    wl = ikpso.workload(1)
    rng = oracle.init_generators(wl.particles, 0)
    f0 = oracle.fitness(wl.chain, ikpso.reference_scene().origin.to_coords())
    res, _, bests = oracle.calculate_pso(wl.chain, wl.particles, rng, iterations=wl.iterations)
    assert bests.min() < 0.5 * f0
    assert oracle.residual(wl.chain, res) < oracle.residual(wl.chain, ikpso.reference_scene().origin.to_coords())
