"""The tip-backward evaluation of the FAST serial-chain kernels
(csrc/ikpso_device.h: TipBackAcc, TipBackAccDH) rests on one identity: for a
chain whose only position term is the tip, the forward frame composition of the
reference's FK (src/kernel.cu:52-56,160-187: W_k = W_{k-1} R_k,
p_k = p_{k-1} + len_k W_k e_x) and the Horner form evaluated from the tip back

    p_J = p_0 + R_0 (R_1 (l_1 e_x + R_2 (l_2 e_x + ... R_J (l_J e_x))))

give the same point.  Checked here in float64 with the kernels' own plane
rotation order (Rz, then Ry, then Rx applied to one vector), for the Euler chain
and for the folded chain (W_j = W_{j-1} C_j Rz(t_j), q_j = q_{j-1} + W_j s_j).
The device kernels' fp32 results are compared with the oracle on the GPU
(tests/test_gpu_parity.py::test_config5_chain_with_penalty, test_gpu_fullsize.py,
test_gpu_mask.py)."""
import numpy as np


def rx(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def ry(b):
    c, s = np.cos(b), np.sin(b)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def rz(t):
    c, s = np.cos(t), np.sin(t)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def euler_forward(R0, p0, ang, lens):
    W, p = R0, p0.copy()
    for (a, b, c), l in zip(ang, lens):
        W = W @ rx(a) @ ry(b) @ rz(c)
        p = p + l * W[:, 0]
    return p


def euler_backward(R0, p0, ang, lens):
    """TipBackAcc::back, node J down to 1, then finish()."""
    u = np.zeros(3)
    J = len(lens)
    for k in range(J, 0, -1):
        a, b, c = ang[k - 1]
        sa, ca, sb, cb, sc, cc = np.sin(a), np.cos(a), np.sin(b), np.cos(b), np.sin(c), np.cos(c)
        l = lens[k - 1]
        if k == J:
            w0, w1, w2 = cc * l, sc * l, 0.0
        else:
            a0 = u[0] + l
            w0, w1, w2 = cc * a0 - sc * u[1], sc * a0 + cc * u[1], u[2]
        y0, y2 = cb * w0 + sb * w2, cb * w2 - sb * w0
        u = np.array([y0, ca * w1 - sa * y2, sa * w1 + ca * y2])
    return p0 + R0 @ u


def test_euler_chain_tip_backward_equals_forward():
    rng = np.random.default_rng(7)
    for J in (1, 2, 7, 20):
        for _ in range(20):
            R0 = rx(rng.uniform(-3, 3)) @ ry(rng.uniform(-3, 3)) @ rz(rng.uniform(-3, 3))
            p0 = rng.uniform(-1, 1, 3)
            ang = rng.uniform(0, 2 * np.pi, (J, 3))
            lens = rng.uniform(0.0, 1.0, J)
            want = euler_forward(R0, p0, ang, lens)
            got = euler_backward(R0, p0, ang, lens)
            assert np.max(np.abs(got - want)) < 1e-12


def test_folded_chain_tip_backward_equals_forward():
    rng = np.random.default_rng(8)
    for J in (3, 7, 12):
        for _ in range(20):
            C = [rx(rng.uniform(-3, 3)) @ ry(rng.uniform(-3, 3)) @ rz(rng.uniform(-3, 3)) for _ in range(J)]
            s = rng.uniform(-0.5, 0.5, (J, 3))
            q0 = rng.uniform(-1, 1, 3)
            t = rng.uniform(-3, 3, J)
            # forward (FitnessAccDH::advance_sc)
            W, q = np.eye(3), q0.copy()
            for j in range(J):
                W = W @ C[j] @ rz(t[j])
                q = q + W @ s[j]
            # backward (TipBackAccDH::back): u <- C_k Rz(t_k) (s_k + u)
            u = np.zeros(3)
            for k in range(J, 0, -1):
                w = s[k - 1] + (u if k < J else 0.0)
                u = C[k - 1] @ (rz(t[k - 1]) @ w)
            assert np.max(np.abs(q0 + u - q)) < 1e-12
