"""Collider term on the GPU (ikpso_collide.h) vs the oracle's GJK restatement
(oracle/ikpso_gjk.c), through the C ABI.

Tolerances: the collision decision is integer-like (hit -> FLT_MAX), so in
REFERENCE arithmetic (the reference's FK operation order and GJK on both sides)
the fitness of every pose and the whole calculatePSO state are compared bit for
bit.  FAST arithmetic tests the boxes by separating axes (ikpso_collide.h:
obb_overlap, round 6) on frames that differ by FMA rounding (<= 2e-5), where the
reference runs GJK, whose tolerance also counts boxes within ~3.5e-4 of touching:
decisions may flip only for boxes that close to touching -- >= 99% of decisions
must agree and finite fitness values meet the FAST FK tolerance; whole FAST solves
are held to the stated tier-B tests against the oracle (test_collide_leg_tier_b).
"""
import numpy as np
import pytest

import ikpso

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

FMAX = np.float32(np.finfo(np.float32).max)


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


@pytest.fixture(scope="module")
def scene_chain():
    return ikpso.reference_scene(reset=True).origin.to_cuda()


def random_colliders(rng, n):
    c = np.zeros(n, dtype=ikpso.COLLIDER_DTYPE)
    for i in range(n):
        q = rng.normal(size=4)
        c[i]["x"], c[i]["y"], c[i]["z"] = rng.uniform(0.2, 1.2, 3)
        c[i]["pos"] = rng.uniform(-2.5, 2.5, 3)
        c[i]["quat"] = q / np.linalg.norm(q)
    return c


@pytest.mark.parametrize("arith", ["reference", "fast"])
def test_evaluate_with_colliders(oracle, device, scene_chain, arith):
    rng = np.random.default_rng(11)
    n = 3000
    ang = rng.uniform(0, 2 * np.pi, (n, 21)).astype(np.float32)
    for boxes in (ikpso.init_colliders(4), random_colliders(rng, 3)):
        s = ikpso.BatchSolver(scene_chain, 64, arith=arith, colliders=boxes)
        fit = s.evaluate(dev(ang))[0].cpu().numpy()
        s.close()
        ofit = np.array([oracle.fitness(scene_chain, a, colliders=boxes) for a in ang], dtype=np.float32)
        hit, ohit = fit == FMAX, ofit == FMAX
        assert 0.05 < ohit.mean() < 0.95  # both outcomes exercised
        if arith == "reference":
            assert np.array_equal(fit, ofit)
        else:
            assert np.mean(hit == ohit) >= 0.99
            both = ~hit & ~ohit
            assert np.max(np.abs(fit[both] - ofit[both]) / ofit[both]) < 1e-5


def run_compat(chain, P, I, colliders, seed_base=0):
    D = 3 * (chain.shape[0] - 1)
    parts = ikpso.particles_tensor(P, D)
    bests = torch.zeros(P, dtype=torch.float32, device="cuda")
    r = ikpso.rng_tensor(P)
    assert ikpso.init_generators_seeded(r, P, seed_base) == 0
    res = np.zeros(D, dtype=np.float32)
    st = ikpso.calculate_pso(parts, None, bests, r, P, chain, ikpso.PSOConfig(0.5, 0.5, 1.25, I),
                             ikpso.FitnessConfig(3.0, 0.0, 0.1), res, colliders, len(colliders))
    assert st == 0
    return res, parts.cpu().numpy(), bests.cpu().numpy(), r.cpu().numpy()


@pytest.mark.parametrize("kernel,P,I", [("resident", 256, 20), ("streaming", 600, 8), ("coop", 2048, 6),
                                      ("auto", 4096, 4)])
def test_calculate_pso_with_colliders_reference_bitexact(oracle, device, scene_chain, monkeypatch, kernel, P, I):
    """calculatePSO(..., colliders, colliderCount) with colliders 0 and 3 of
    initColliders (1 and 2 intersect the reset pose), REFERENCE arithmetic."""
    monkeypatch.setenv("IKPSO_ARITH", "reference")
    if kernel != "auto":  # auto: a single swarm of 4096 takes the cooperative latency variant
        monkeypatch.setenv("IKPSO_KERNEL", kernel)
    else:
        monkeypatch.delenv("IKPSO_KERNEL", raising=False)
    boxes = ikpso.init_colliders(4)[[0, 3]]
    res, parts, bests, r = run_compat(scene_chain, P, I, boxes)
    ostate = oracle.init_generators(P, 0)
    ores, oparts, obests = oracle.calculate_pso(scene_chain, P, ostate, iterations=I, colliders=boxes)
    assert np.array_equal(r[:, :6], ostate.view(np.int32).reshape(P, 12)[:, :6])
    assert np.array_equal(bests, obests) and np.array_equal(parts, oparts) and np.array_equal(res, ores)
    assert oracle.fitness(scene_chain, res, colliders=boxes) < FMAX
    # the term changed the run: without colliders the local bests differ
    _, _, nobests = oracle.calculate_pso(scene_chain, P, oracle.init_generators(P, 0), iterations=I)
    assert not np.array_equal(nobests, obests)


def test_batch_with_colliders_fast(oracle, device):
    """Batched FAST solve with a collider between the arm and its targets:
    every swarm's answer is collision-free and its fitness matches the oracle's
    statistically (tier B)."""
    wl = ikpso.workload(3)
    B, P, I = 32, 256, 40
    boxes = np.concatenate([ikpso.make_collider((0.6, 0.6, 0.6), (0.0, 0.9, -1.6)), ikpso.init_colliders(1)])
    tg = wl.targets(0, B)
    s = ikpso.BatchSolver(wl.chain, P, pso=wl.pso, colliders=boxes)
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    # the device's own evaluation of its answers: collision-free, same fitness
    efit = s.evaluate(dev(ang), dev(tg))[0].cpu().numpy()
    s.close()
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, ores = oracle.solve_batch(wl.chain, tg, None, P, I, ostate, colliders=boxes, threads=8)
    assert (fit < FMAX).all() and (ofit < FMAX).all() and np.array_equal(efit, fit)
    # PSO drives answers onto the obstacle's surface, so a FAST answer may touch
    # it within FMA rounding of the reference-order FK; against colliders shrunk
    # by 1% (3 mm on a 0.6 box) every answer must be clear
    shrunk = boxes.copy()
    for ax in ("x", "y", "z"):
        shrunk[ax] *= 0.99
    clear = [oracle.fitness(_with_targets(wl.chain, tg[b]), ang[b], colliders=shrunk) < FMAX for b in range(B)]
    assert all(clear), clear
    assert abs(fit.mean() - ofit.mean()) / ofit.mean() < 0.02


def _with_targets(chain, tg):
    ch = chain.copy()
    ch["target_position"][5:8] = tg
    return ch


def test_long_chain_colliders_cooperative(oracle, device):
    """A 12-joint serial chain (D = 36) with colliders solved by the cooperative
    kernel: its collider build needs more than 256 VGPRs, so it cannot run the two
    workgroups per CU the long-chain geometry plans; the launch fits the
    concurrent groups to the build's real occupancy (one per CU) instead of
    failing.  REFERENCE arithmetic: bit-exact to the oracle."""
    chain = ikpso.serial_chain(12, length=0.4).to_cuda()
    boxes = ikpso.init_colliders(2)
    B, P, I = 3, 1024, 6
    rng = np.random.default_rng(23)
    tg = rng.uniform(-2.0, 2.0, (B, 1, 3)).astype(np.float32)
    s = ikpso.BatchSolver(chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith="reference", kernel="coop",
                          colliders=boxes)
    assert "coop" in s.kernel and "serial_tip12" in s.kernel
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    assert s.fallbacks == 0
    s.close()
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, ores = oracle.solve_batch(chain, tg, None, P, I, ostate, colliders=boxes, threads=4)
    assert np.array_equal(ang, oang) and np.array_equal(fit, ofit)


@pytest.mark.parametrize("scene,masked", [("all4", False), ("013", False), ("013", True)])
def test_resident_full_swarm_colliders_reference_bitexact(oracle, device, scene, masked):
    """The resident collider build at its full 1024 lanes -- the velocities of
    dimensions 0-17 held in LDS behind the local bests (kVelLds) -- with boxes that
    the arm reaches: every initColliders box (two intersect the reset pose, so
    evaluations carry several near nodes and many hit: FitnessAcc::finish's loop over
    the stored frames runs several trips and stops at a hit), or boxes 0, 1 and 3;
    unmasked and with an axis mask (the masked collider build).  REFERENCE
    arithmetic: bit-exact to the oracle."""
    wl = ikpso.workload(3)
    boxes = ikpso.init_colliders(4)
    if scene == "013":
        boxes = boxes[[0, 1, 3]]
    mask = np.array([0, 7, 5, 7, 0, 6, 7, 3], np.uint8) if masked else None
    B, P, I = 3, 1024, 8
    tg = wl.targets(0, B)
    s = ikpso.BatchSolver(wl.chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith="reference",
                          kernel="resident", colliders=boxes, axis_mask=mask)
    assert "resident" in s.kernel
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    s.close()
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, ores = oracle.solve_batch(wl.chain, tg, None, P, I, ostate, colliders=boxes, threads=8,
                                          axis_mask=mask)
    assert np.array_equal(ang, oang) and np.array_equal(fit, ofit)


def test_collide_leg_tier_b(oracle, device, report):
    """The bench's collide leg at its own configuration (bench.py collide_leg: config 3's
    targets, 1024 particles x 500 iterations, the reference's initColliders boxes 0 and 3,
    src/Main.cpp:537-559; the term src/kernel.cu:104-136), FAST, on the 256 swarms of
    tests/golden/tierb_collide.npz: the stated tests of tests/tierb.py against the oracle's
    FMA on/off envelope (Fisher tests of the shares with the absolute floor, strict sign test
    of the fitness, alpha = 0.01), gross-error ceilings at twice the envelope's worst swarm,
    mean fitness within 0.5 %, every answer collision-free with the device's own evaluation
    of it equal to the reported fitness, generator states bit-exact.  This covers the
    improving-lanes filter (ikpso_collide.h: only lanes whose collision-free value could
    pass the strict local-best update run GJK) over whole FAST solves."""
    from tierb import envelope, load_fixture, stat_tests, tier_b_distances, tier_b_report

    wl = ikpso.workload(3)
    fx = load_fixture("collide")
    boxes = ikpso.init_colliders(4)[[0, 3]]
    B, P, I, D = int(fx["swarms"]), wl.particles, wl.iterations, wl.dof
    tg = wl.targets(0, B)
    s = ikpso.BatchSolver(wl.chain, P, pso=wl.pso, colliders=boxes)
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    assert "resident" in s.kernel, s.kernel
    efit = s.evaluate(dev(ang), dev(tg))[0].cpu().numpy()
    states = s.generator_states(0, B)
    s.close()
    want = oracle.skipahead(oracle.init_generators(B * P, 0), D + 3 * D * I)
    assert np.array_equal(states[:, :6], want.view(np.int32).reshape(-1, 12)[:, :6])
    assert (fit < FMAX).all() and np.isfinite(ang).all()
    assert np.array_equal(efit, fit)  # one arithmetic: the solve's fitness is the evaluate kernel's
    env = envelope(wl.chain, fx)
    rang, rfit, rres = fx["ref_angles"], fx["ref_fitness"], fx["ref_residual"]
    dist = tier_b_distances(wl.chain, ang, fit, res, rang, rfit, rres)
    rep = tier_b_report(*dist)
    tests = stat_tests(dist, env, fit, rfit)
    rep.update(mean_fitness=float(fit.mean()), oracle_mean_fitness=float(rfit.mean()), envelope=tier_b_report(*env),
               tests=tests)
    report("tier_b_collide", rep)
    assert tests["pass"], tests
    for d, e in zip(dist, env):
        assert d.max() <= 2 * e.max(), (d.max(), e.max())
    assert abs(fit.mean() - rfit.mean()) / rfit.mean() < 5e-3
    assert abs(res.mean() - rres.mean()) < 1e-3 + 0.01 * rres.mean()
    # the oracle's own verdict on the answers: clear of the boxes (within FMA rounding of the
    # reference-order FK: against boxes shrunk by 1 %)
    shrunk = boxes.copy()
    for ax in ("x", "y", "z"):
        shrunk[ax] *= 0.99
    assert all(oracle.fitness(_with_targets(wl.chain, tg[b]), ang[b], colliders=shrunk) < FMAX for b in range(B))


@pytest.mark.parametrize("kernel", ["resident", "auto"])
def test_collide_leg_reference_whole_solve(oracle, device, kernel):
    """REFERENCE arithmetic over whole solves of the collide leg (500 iterations), the first
    8 swarms of tests/golden/tierb_collide.npz, on the resident kernel and (AUTO: few swarms)
    the cooperative latency variant: angles and fitness bit-identical to the oracle's, so
    the improving-lanes filter changes no decision over a full solve."""
    from tierb import load_fixture

    wl = ikpso.workload(3)
    fx = load_fixture("collide")
    boxes = ikpso.init_colliders(4)[[0, 3]]
    B, P, I = 8, wl.particles, wl.iterations
    s = ikpso.BatchSolver(wl.chain, P, pso=wl.pso, arith="reference", colliders=boxes, kernel=kernel)
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(wl.targets(0, B)), iterations=I))
    assert ("latency variant" in s.kernel) == (kernel == "auto"), s.kernel
    s.close()
    assert np.array_equal(ang, fx["ref_angles"][:B]) and np.array_equal(fit, fx["ref_fitness"][:B])
    assert np.max(np.abs(res - fx["ref_residual"][:B])) <= 1e-5


@pytest.mark.parametrize("arith", ["reference", "fast"])
def test_far_colliders_skip_the_term(oracle, device, monkeypatch, arith):
    """Host-side pruning (parse_chain): colliders beyond the arm's reach of every node
    (the reference's four initColliders boxes moved 1000 units away) can never pass the
    inline sphere test, so the solver leaves them out -- with none left it drops the term
    and runs the plain kernels; a far box beside near ones is left out alone (REFERENCE:
    bit-exact to the oracle with all three).
    REFERENCE: bit-exact to the oracle with the colliders (its GJK runs and finds nothing)
    and to the same solver kept on the collider kernel (IKPSO_KEEP_FAR_COLLIDERS=1).
    FAST: bit-identical to a solver without colliders; a box within reach keeps the term."""
    wl = ikpso.workload(3)
    far = ikpso.init_colliders(4)
    far["pos"] += 1000.0
    B, P, I = 4, 1024, 12
    tg = wl.targets(0, B)

    def solve(boxes):
        s = ikpso.BatchSolver(wl.chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith=arith, colliders=boxes)
        n = s.collider_count
        s.seed(B)
        out = [t.cpu().numpy() for t in s.solve(dev(tg), iterations=I)]
        s.close()
        return n, out

    monkeypatch.delenv("IKPSO_KEEP_FAR_COLLIDERS", raising=False)
    n_far, (ang, fit, res) = solve(far)
    assert n_far == 0
    n_none, (ang0, fit0, res0) = solve(None)
    assert n_none == 0 and np.array_equal(ang, ang0) and np.array_equal(fit, fit0)
    near = ikpso.init_colliders(4)[[0, 3]]
    assert solve(near)[0] == 2
    # a box just beyond the reach bound is dropped, one just inside kept
    arm = float(np.abs(wl.chain["length"][1:]).sum())
    edge = ikpso.make_collider((0.2, 0.2, 0.2), (arm + 2.0, 0.0, 0.0))
    assert solve(edge)[0] == 0
    edge["pos"][0] = (arm, 0.0, 0.0)
    assert solve(edge)[0] == 1
    # a far box beside near ones is left out alone
    mixed = np.concatenate([near, far[:1]])
    n_mixed, (angm, fitm, _) = solve(mixed)
    assert n_mixed == 2
    if arith == "reference":
        ostate = oracle.init_generators(B * P, 0)
        oang, ofit, ores = oracle.solve_batch(wl.chain, tg, None, P, I, ostate, colliders=far, threads=8)
        assert np.array_equal(ang, oang) and np.array_equal(fit, ofit)
        ostate = oracle.init_generators(B * P, 0)
        oang, ofit, ores = oracle.solve_batch(wl.chain, tg, None, P, I, ostate, colliders=mixed, threads=8)
        assert np.array_equal(angm, oang) and np.array_equal(fitm, ofit)
        monkeypatch.setenv("IKPSO_KEEP_FAR_COLLIDERS", "1")
        n_keep, (angk, fitk, _) = solve(far)
        assert n_keep == 4 and np.array_equal(angk, ang) and np.array_equal(fitk, fit)
