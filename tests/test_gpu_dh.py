"""DH arms and the opt-in distance-term slot fix on the GPU, through the C ABI.

REFERENCE arithmetic is compared with the oracle bit for bit (the DH front-end
only builds a node table, so the reference's own algorithm applies); FAST
solves are checked on what an IK user needs: reachable targets are reached.
"""
import numpy as np
import pytest

import ikpso
from ikpso.dh import dh_arm, dh_forward

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

IIWA = dict(a=[0.0] * 7, alpha=[-np.pi / 2, np.pi / 2, np.pi / 2, -np.pi / 2, -np.pi / 2, np.pi / 2, 0.0],
            d=[0.36, 0.0, 0.42, 0.0, 0.4, 0.0, 0.126])
LIM = np.radians([170, 120, 170, 120, 170, 120, 175])
# an arm with every offset along the links (d = 0): one node per joint
PLANARISH = dict(a=[0.4, 0.35, 0.3, 0.25, 0.2, 0.15, 0.1], alpha=[np.pi / 2, -np.pi / 2] * 3 + [0.0], d=[0.0] * 7)


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def reachable_targets(arm_spec, n, rng):
    th = rng.uniform(-0.8, 0.8, (n, 7)) * LIM
    return np.array([dh_forward(t, arm_spec["d"], arm_spec["a"], arm_spec["alpha"]) for t in th], np.float32)


@pytest.mark.parametrize("spec,kern,P", [(IIWA, "serial_tip11", 256), (PLANARISH, "serial_tip7", 256),
                                         (PLANARISH, "serial_tip7", 1024)])
def test_dh_reference_bitexact(oracle, device, spec, kern, P):
    """REFERENCE, bit-exact to the oracle.  The 7-joint arm's swarms take the
    cooperative latency variant with generator waves: one chunk at P = 256, four
    at P = 1024."""
    arm = dh_arm(spec["a"], spec["alpha"], spec["d"], -LIM, LIM)
    chain = arm.origin.to_cuda()
    rng = np.random.default_rng(5)
    B, I = 4, 12
    tg = reachable_targets(spec, B, rng).reshape(B, 1, 3)
    s = ikpso.BatchSolver(chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith="reference")
    assert kern in s.kernel
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    s.close()
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, ores = oracle.solve_batch(chain, tg, None, P, I, ostate, threads=4)
    assert np.array_equal(ang, oang) and np.array_equal(fit, ofit)
    assert np.max(np.abs(res - ores)) < 1e-5


@pytest.mark.parametrize("spec", [IIWA, PLANARISH])
def test_dh_solves_reachable_targets(device, spec):
    """FAST, 1024 particles, 400 iterations: the tool reaches reachable targets."""
    arm = dh_arm(spec["a"], spec["alpha"], spec["d"], -LIM, LIM)
    chain = arm.origin.to_cuda()
    rng = np.random.default_rng(9)
    B = 64
    tg = reachable_targets(spec, B, rng)
    fit_cfg = ikpso.FitnessConfig(0.0, 0.0, 0.1)  # position only: no pull towards the rest pose
    s = ikpso.BatchSolver(chain, 1024, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, 400), fit=fit_cfg)
    # 7 nodes: one workgroup per swarm; 11 nodes (iiwa: 4 d offsets): four 256-lane chunks per swarm
    assert ("resident" if len(chain) == 8 else "coop") in s.kernel
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg.reshape(B, 1, 3)), iterations=400))
    s.close()
    # check through the textbook DH product, not the solver's own FK
    tool = np.array([dh_forward(arm.joint_angles(a), spec["d"], spec["a"], spec["alpha"]) for a in ang])
    err = np.linalg.norm(tool - tg, axis=1)
    assert np.allclose(err, res, atol=1e-4)
    assert np.median(err) < 1e-3 and np.mean(err < 1e-2) >= 0.9, err
    th = np.array([arm.joint_angles(a) for a in ang])
    assert np.all(np.abs(th) <= LIM + 1e-5)  # joint limits hold


def test_posref_node_slot_flag(oracle, device):
    """IKPSO_FLAG_POSREF_NODE_SLOT: node k reads positions slot k+1 (FillPositions'
    own slot); equivalent to the reference's reading of positions[8:]."""
    sc = ikpso.reference_scene(reset=True)
    chain = sc.origin.to_cuda()
    positions = sc.origin.fill_positions()            # [4 * (J + 2)]
    assert positions.size == 4 * 9
    fit_cfg = ikpso.FitnessConfig(3.0, 1.0, 0.1)
    B, P, I = 2, 256, 10
    tg = np.repeat(ikpso.RESET_TARGETS[None], B, axis=0)
    out = {}
    for flag in (False, True):
        s = ikpso.BatchSolver(chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), fit=fit_cfg, arith="reference",
                              positions=positions, posref_node_slot=flag)
        s.seed(B)
        out[flag] = [t.cpu().numpy() for t in s.solve(dev(tg), iterations=I)]
        s.close()
    for flag, pos in ((False, positions[:28]), (True, positions[8:])):
        ostate = oracle.init_generators(B * P, 0)
        oang, ofit, _ = oracle.solve_batch(chain, tg, None, P, I, ostate, distance_weight=1.0, positions=pos)
        assert np.array_equal(out[flag][0], oang) and np.array_equal(out[flag][1], ofit), flag
    assert not np.array_equal(out[False][1], out[True][1])
