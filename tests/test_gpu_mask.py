"""Joint-axis masks and the folded serial chain on the GPU, through the C ABI
(extension: SURVEY.md §8(f) row 4; the reference hard-wires 3 Euler axes per
node, src/kernel.cu:52-56,160-187).

Semantics (oracle/ikpso_oracle.c, orc_solve_batch_mask): a locked angle stays
at its node's rotation -- no draws, no update, no clamp -- and D is the number
of free angles; the fitness is the reference's calculateDistance of the full
Euler vector.

  * REFERENCE arithmetic runs the Euler kernels with the mask: bit for bit
    equal to the oracle (resident, cooperative and streaming families).
  * FAST solves of a masked serial chain with a tip effector run on the folded
    chain (TopoDH: one sincos per free angle).  Its FK rounds differently from
    the Euler form, so it is held to the FAST tolerances of test_gpu_parity.py:
    one pose |df|/f <= 1e-5 and tip |dp| <= 2e-5; tier A |dtheta| <= 1e-4 rad
    and |df|/f <= 1e-5.  Tier A compares angles at I = 5 on this arm and the
    fitness up to I = 20: the oracle against itself with FMA contraction on/off
    (tests/test_oracle_divergence.py) agrees to 2.4e-7 rad at I = 10 but
    drifts to 4.3e-4 rad at I = 20 on the iiwa (the reference scene: 4.8e-7 at
    I = 20), and the folded FK differs from the oracle's 4x4 products by more
    than one FMA rounding (fp32-rounded fold constants, hardware sin/cos within
    5e-7), so with 12k particles a pbest acceptance can flip by I = 10; the
    fitness stays within 1e-5 throughout.  Tier B: folded vs unfolded at I = 300.
"""
import numpy as np
import pytest

import ikpso
from ikpso import _abi
from ikpso.dh import dh_arm, dh_forward

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

IIWA = dict(a=[0.0] * 7, alpha=[-np.pi / 2, np.pi / 2, np.pi / 2, -np.pi / 2, -np.pi / 2, np.pi / 2, 0.0],
            d=[0.36, 0.0, 0.42, 0.0, 0.4, 0.0, 0.126])
LIM = np.radians([170, 120, 170, 120, 170, 120, 175])


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def iiwa():
    return dh_arm(IIWA["a"], IIWA["alpha"], IIWA["d"], -LIM, LIM)


def reachable(n, rng):
    th = rng.uniform(-0.8, 0.8, (n, 7)) * LIM
    return np.array([dh_forward(t, IIWA["d"], IIWA["a"], IIWA["alpha"]) for t in th], np.float32)


def solve(chain, mask, tg, P, I, arith, kernel="auto", fold=True, start=None, **kw):
    s = ikpso.BatchSolver(chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith=arith, kernel=kernel,
                          axis_mask=mask, fold=fold, **kw)
    B = tg.shape[0]
    s.seed(B)
    out = [t.cpu().numpy() for t in s.solve(dev(tg), iterations=I,
                                            start_pose=None if start is None else dev(start))]
    name, dof = s.kernel, s.dof
    s.close()
    return out, name, dof


# --------------------------------------------------------- REFERENCE: bit-exact
@pytest.mark.parametrize("kernel,P", [("resident", 256), ("coop", 1024), ("streaming", 300)])
def test_masked_dh_arm_reference_bitexact(oracle, device, kernel, P):
    """iiwa as 11 reference nodes, only the 7 joint z angles free (D = 7)."""
    arm = iiwa()
    chain, mask = arm.origin.to_cuda(), arm.axis_mask
    rng = np.random.default_rng(3)
    B, I = 4, 12
    tg = reachable(B, rng).reshape(B, 1, 3)
    (ang, fit, res), name, dof = solve(chain, mask, tg, P, I, "reference", kernel)
    assert dof == 7 and ang.shape == (B, 7) and kernel in name and "serial_tip11" in name
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, ores = oracle.solve_batch(chain, tg, None, P, I, ostate, threads=4, axis_mask=mask)
    assert np.array_equal(ang, oang) and np.array_equal(fit, ofit)
    assert np.max(np.abs(res - ores)) < 1e-5


@pytest.mark.parametrize("kernel", ["resident", "streaming"])
def test_masked_reference_scene_bitexact(oracle, device, kernel):
    """The reference's 7-node tree with a random mask, a per-swarm start pose and
    the soft-limit penalty over the free angles."""
    wl = ikpso.workload(3)
    rng = np.random.default_rng(11)
    mask = np.concatenate([[0], rng.integers(1, 8, 7)]).astype(np.uint8)
    mask[3] = 0  # a fully locked node
    D = int(sum(bin(m).count("1") for m in mask[1:]))
    B, P, I = 3, 256, 10
    tg = wl.targets(0, B)
    start = rng.uniform(0.5, 2.5, (B, D)).astype(np.float32)
    lo, hi = np.full(D, 0.8, np.float32), np.full(D, 2.0, np.float32)
    (ang, fit, res), name, dof = solve(wl.chain, mask, tg, P, I, "reference", kernel, start=start,
                                       limit_weight=10.0, soft_lo=lo, soft_hi=hi)
    assert dof == D and "ref_tree7" in name
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, ores = oracle.solve_batch(wl.chain, tg, start, P, I, ostate, threads=4, axis_mask=mask,
                                          limit_weight=10.0, soft_lo=lo, soft_hi=hi)
    assert np.array_equal(ang, oang) and np.array_equal(fit, ofit)
    assert np.max(np.abs(res - ores)) < 1e-5


def test_masked_generic_tree_reference_bitexact(oracle, device):
    """A branching tree (generic topology kernels) with a mask and the distance term."""
    sc = ikpso.reference_scene(reset=True)
    chain = sc.origin.to_cuda().copy()
    chain["parent_index"][5] = 2  # re-hang one wrist: no longer the reference tree
    mask = np.array([0, 7, 1, 2, 4, 5, 6, 3], np.uint8)
    D = int(sum(bin(m).count("1") for m in mask[1:]))
    B, P, I = 2, 200, 8
    tg = np.repeat(ikpso.RESET_TARGETS[None], B, axis=0)
    positions = sc.origin.fill_positions()[:28]
    s = ikpso.BatchSolver(chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith="reference",
                          fit=ikpso.FitnessConfig(3.0, 1.0, 0.1), positions=positions, axis_mask=mask)
    assert "generic" in s.kernel and s.dof == D
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    s.close()
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, _ = oracle.solve_batch(chain, tg, None, P, I, ostate, threads=4, axis_mask=mask,
                                       distance_weight=1.0, positions=positions)
    assert np.array_equal(ang, oang) and np.array_equal(fit, ofit)


def test_masked_evaluate_matches_oracle(oracle, device):
    """evaluate() of a masked solver places the D free angles and keeps the
    locked ones at rest (REFERENCE: bit for bit)."""
    arm = iiwa()
    chain, mask = arm.origin.to_cuda(), arm.axis_mask
    rng = np.random.default_rng(8)
    n = 64
    ang = (rng.uniform(-1, 1, (n, 7)) * LIM + arm.z_offset).astype(np.float32)
    tg = reachable(n, rng).reshape(n, 1, 3)
    s = ikpso.BatchSolver(chain, 64, arith="reference", axis_mask=mask)
    fit, pos = (t.cpu().numpy() for t in s.evaluate(dev(ang), dev(tg)))
    s.close()
    for i in range(0, n, 7):
        c = chain.copy()
        c["target_position"][-1] = tg[i, 0]
        assert fit[i] == oracle.fitness_mask(c, ang[i], mask)
    # tool position = the textbook DH product of the joint angles
    tool = np.array([dh_forward(arm.joint_angles(a), IIWA["d"], IIWA["a"], IIWA["alpha"]) for a in ang])
    assert np.max(np.abs(pos.reshape(n, -1, 3)[:, -1] - tool)) < 2e-5


def test_mask_validation(device):
    arm = iiwa()
    chain = arm.origin.to_cuda()
    for bad in (np.zeros(len(chain), np.uint8), np.full(len(chain), 9, np.uint8)):
        with pytest.raises(_abi.IkpsoError):
            ikpso.BatchSolver(chain, 64, axis_mask=bad)
    with pytest.raises(ValueError):
        ikpso.BatchSolver(chain, 64, axis_mask=np.ones(3, np.uint8))


# ------------------------------------------------------- FAST: the folded chain
def test_folded_chain_one_pose(oracle, device):
    """I = 0 with a random start pose per swarm: the reported fitness is the
    folded FK's fitness of that pose, within the FAST one-pose tolerance; the
    residual is the tip distance."""
    arm = iiwa()
    chain, mask = arm.origin.to_cuda(), arm.axis_mask
    rng = np.random.default_rng(21)
    B = 64
    tg = reachable(B, rng).reshape(B, 1, 3)
    start = (rng.uniform(-1, 1, (B, 7)) * LIM + arm.z_offset).astype(np.float32)
    (ang, fit, res), name, _ = solve(chain, mask, tg, 64, 0, "fast", start=start)
    assert "dh7" in name
    np.testing.assert_array_max_ulp(ang, start, 4)  # the start pose through revolutions (kTermRev)
    fd = oracle.free_dims(chain, mask)
    for b in range(B):
        c = chain.copy()
        c["target_position"][-1] = tg[b, 0]
        rot = c["rotation"][1:].reshape(-1)
        rot[fd] = start[b]  # the start pose is the angle term's reference
        c["rotation"][1:] = rot.reshape(-1, 3)
        ofit = float(oracle.fitness_mask(c, start[b], mask))  # angle term 0: fitness = |tip - t|^2
        assert abs(fit[b] - ofit) <= 1e-5 * ofit + 1e-10
        tip = dh_forward(arm.joint_angles(start[b]), IIWA["d"], IIWA["a"], IIWA["alpha"])
        assert abs(res[b] - np.linalg.norm(tip - tg[b, 0])) < 2e-5


@pytest.mark.parametrize("kernel,P", [("resident", 1024), ("auto", 1024), ("coop", 2048), ("streaming", 600)])
def test_folded_chain_tier_a(oracle, device, kernel, P):
    """Tier A (I = 20) against the oracle's masked solve on the same seeds."""
    arm = iiwa()
    chain, mask = arm.origin.to_cuda(), arm.axis_mask
    rng = np.random.default_rng(5)
    B = 6
    tg = reachable(B, rng).reshape(B, 1, 3)
    for I in (5, 10, 20):
        (ang, fit, res), name, dof = solve(chain, mask, tg, P, I, "fast", kernel)
        assert "dh7" in name and dof == 7
        ostate = oracle.init_generators(B * P, 0)
        oang, ofit, ores = oracle.solve_batch(chain, tg, None, P, I, ostate, threads=8, axis_mask=mask)
        assert np.max(np.abs(fit - ofit) / ofit) < 1e-5
        if I == 5:
            assert np.max(np.abs(ang - oang)) < 1e-4
            assert np.max(np.abs(res - ores)) < 1e-4


def test_folded_chain_with_penalty_and_bounds(oracle, device):
    """Uniform bounds and the soft-limit penalty (the other folded builds)."""
    arm = iiwa()
    chain, mask = arm.origin.to_cuda().copy(), arm.axis_mask
    rng = np.random.default_rng(13)
    B, P, I = 4, 512, 5
    tg = reachable(B, rng).reshape(B, 1, 3)
    lo, hi = -0.6 * LIM.astype(np.float32), 0.6 * LIM.astype(np.float32)
    (ang, fit, res), name, _ = solve(chain, mask, tg, P, I, "fast", limit_weight=10.0,
                                     soft_lo=lo + arm.z_offset, soft_hi=hi + arm.z_offset)
    assert "dh7" in name
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, _ = oracle.solve_batch(chain, tg, None, P, I, ostate, threads=4, axis_mask=mask,
                                       limit_weight=10.0, soft_lo=lo + arm.z_offset, soft_hi=hi + arm.z_offset)
    assert np.max(np.abs(ang - oang)) < 1e-4
    assert np.max(np.abs(fit - ofit) / ofit) < 1e-5


def test_folded_equals_unfolded_statistically(device):
    """FAST folded vs FAST Euler-with-mask (IKPSO_FLAG_NO_FOLD) at I = 300: the
    same answers up to chaos -- tier B over 64 swarms."""
    arm = iiwa()
    chain, mask = arm.origin.to_cuda(), arm.axis_mask
    rng = np.random.default_rng(17)
    B, P, I = 64, 256, 300
    tg = reachable(B, rng).reshape(B, 1, 3)
    pos_only = ikpso.FitnessConfig(0.0, 0.0, 0.1)
    (a1, f1, r1), n1, _ = solve(chain, mask, tg, P, I, "fast", fit=pos_only)
    (a2, f2, r2), n2, _ = solve(chain, mask, tg, P, I, "fast", fold=False, fit=pos_only)
    assert "dh7" in n1 and "serial_tip11" in n2
    assert np.median(r1) < 1e-2 and np.median(r2) < 1e-2
    assert abs(np.mean(r1 < 1e-2) - np.mean(r2 < 1e-2)) <= 0.1


def test_dh_arm_masked_solves_reachable_targets(device):
    """The DH front-end's use case, masked and folded: 7 free angles, the tool
    reaches reachable targets (checked through the textbook DH product)."""
    arm = iiwa()
    chain, mask = arm.origin.to_cuda(), arm.axis_mask
    rng = np.random.default_rng(9)
    B = 64
    tg = reachable(B, rng)
    fit_cfg = ikpso.FitnessConfig(0.0, 0.0, 0.1)  # position only
    s = ikpso.BatchSolver(chain, 1024, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, 400), fit=fit_cfg, axis_mask=mask)
    assert "dh7" in s.kernel and s.dof == 7
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg.reshape(B, 1, 3)), iterations=400))
    s.close()
    tool = np.array([dh_forward(arm.joint_angles(a), IIWA["d"], IIWA["a"], IIWA["alpha"]) for a in ang])
    err = np.linalg.norm(tool - tg, axis=1)
    assert np.allclose(err, res, atol=1e-4)
    assert np.median(err) < 1e-3 and np.mean(err < 1e-2) >= 0.9, err
    th = np.array([arm.joint_angles(a) for a in ang])
    assert np.all(np.abs(th) <= LIM + 1e-5)


def test_dh7_bench_workload_tier_b(oracle, device):
    """Tier B on the benchmarked DH workload itself (bench.py --config dh7: the
    iiwa arm, reachable targets, position-only fitness, 1024 particles, 500
    iterations), 64 swarms, FAST folded chain vs the oracle's masked Euler solve.
    The oracle drives every swarm's tip onto its target to fp32 resolution
    (residual median 0, max 3.7e-9 on these 64 swarms); so must the GPU: its own
    residual <= 1e-5 on every swarm, and the reference FK (oracle) of its answers
    within 1e-4 of the target (the folded constants are fp32-rounded products, so
    the two FKs of one pose differ by ~1e-6)."""
    wl = ikpso.workload("dh7")
    B, P, I = 64, wl.particles, wl.iterations
    tg = wl.targets(0, B)
    s = ikpso.BatchSolver(wl.chain, P, pso=wl.pso, fit=wl.fit, axis_mask=wl.axis_mask)
    assert "dh7" in s.kernel
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    s.close()
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, ores = oracle.solve_batch(wl.chain, tg, None, P, I, ostate, threads=0, axis_mask=wl.axis_mask,
                                          angle_weight=wl.fit.angle_weight)
    assert ores.max() <= 1e-5
    assert np.isfinite(ang).all() and res.max() <= 1e-5, np.sort(res)[-4:]
    for b in range(B):
        c = wl.chain.copy()
        c["target_position"][-1] = tg[b, 0]
        full = oracle.expand(c, ang[b], wl.axis_mask)
        assert oracle.residual(c, full) <= 1e-4, (b, oracle.residual(c, full))
