"""DH front-end (ikpso/dh.py): a standard-DH arm mapped
onto the reference's node model.  Pinned by the textbook DH product
Rz(theta) Tz(d) Tx(a) Rx(alpha) in float64, through the host node model and
through the oracle's reference-order fp32 FK of the marshalled node table."""
import numpy as np
import pytest

import ikpso
from ikpso.dh import dh_arm, dh_forward

# KUKA LBR iiwa 14-like standard DH table (a = 0, offsets along z)
IIWA = dict(a=[0.0] * 7, alpha=[-np.pi / 2, np.pi / 2, np.pi / 2, -np.pi / 2, -np.pi / 2, np.pi / 2, 0.0],
            d=[0.36, 0.0, 0.42, 0.0, 0.4, 0.0, 0.126])
LIM = np.radians([170, 120, 170, 120, 170, 120, 175])


def random_arm(rng, n=7):
    a = rng.uniform(-0.5, 0.5, n) * (rng.random(n) < 0.6)
    d = rng.uniform(-0.5, 0.5, n) * (rng.random(n) < 0.5)
    al = rng.uniform(-3, 3, n)
    return a, al, d


def test_dh_mapping_matches_textbook_fk(oracle):
    rng = np.random.default_rng(0)
    for _ in range(6):
        a, al, d = random_arm(rng)
        arm = dh_arm(a, al, d, [-3] * 7, [3] * 7)
        chain = arm.origin.to_cuda()
        J = chain.shape[0] - 1
        assert J == 7 + int(np.count_nonzero(d))
        assert chain["parent_index"].tolist() == list(range(-1, J))          # serial
        assert (chain["node_type"][1:] == ikpso.NODE_EFFECTOR).sum() == 1    # tool only
        assert chain["node_type"][-1] == ikpso.NODE_EFFECTOR
        for _ in range(8):
            th = rng.uniform(-3, 3, 7)
            c = arm.coords(th)
            want = dh_forward(th, d, a, al)
            arm.origin.from_coords(c)
            assert np.abs(arm.tool.world_position() - want).max() < 1e-6
            assert np.abs(oracle.node_positions(chain, c)[-1] - want).max() < 2e-5
            assert np.abs(arm.joint_angles(c) - th).max() < 1e-6


def test_dh_locked_axes_and_limits():
    arm = dh_arm(IIWA["a"], IIWA["alpha"], IIWA["d"], -LIM, LIM)
    chain = arm.origin.to_cuda()
    lo, hi = chain["min_rotation"][1:], chain["max_rotation"][1:]
    free = lo != hi
    assert free.sum() == 7                       # one free axis (z) per DH joint
    assert np.all(free[:, :2] == False)          # noqa: E712 -- x, y always locked
    # joint limits survive the offset: hi - lo == 2 * limit on every free axis
    assert np.allclose(np.sort((hi - lo)[free]), np.sort(2 * LIM), atol=1e-6)
    # rest pose = the locked values, so the angle term starts at zero on them
    assert np.array_equal(chain["rotation"][1:][~free], lo[~free])


def test_dh_rejects_bad_tables():
    with pytest.raises(ValueError):
        dh_arm([0.1], [0.0, 0.0], [0.0], [-1], [1])
