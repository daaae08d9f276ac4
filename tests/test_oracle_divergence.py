"""How fast the PSO dynamics amplify an ulp-level FK difference, measured on
the CPU oracle itself: the same restatement built with and without FMA
contraction, same seeds (SURVEY.md §8(c) "Measured divergence").  This sets the
iteration count of the tier-A comparisons: the GPU's FAST arithmetic differs
from the oracle at that level, so tier A is only meaningful while two oracles
that differ by one rounding still agree to well under its 1e-4 rad.

  * reference scene (config 3): FMA on/off agree to < 1e-6 rad at I = 20;
  * the 7-joint iiwa DH arm with its axis mask (D = 7): < 1e-5 rad at I = 10,
    but the angles drift apart by up to ~4e-4 rad at I = 20 while the fitness
    still agrees to ~2e-7 -- so the folded-chain tier A (test_gpu_mask.py) runs
    I = 10 for angles and compares fitness at I = 20.
"""
import ctypes
import subprocess
from pathlib import Path

import numpy as np
import pytest

import ikpso
from ikpso.dh import dh_arm, dh_forward

ROOT = Path(__file__).resolve().parents[1]
IIWA = dict(a=[0.0] * 7, alpha=[-np.pi / 2, np.pi / 2, np.pi / 2, -np.pi / 2, -np.pi / 2, np.pi / 2, 0.0],
            d=[0.36, 0.0, 0.42, 0.0, 0.4, 0.0, 0.126])
LIM = np.radians([170, 120, 170, 120, 170, 120, 175])


@pytest.fixture(scope="module")
def fma_oracle(oracle, tmp_path_factory):
    """The oracle source built with FMA contraction (test-only build)."""
    out = tmp_path_factory.mktemp("ofma") / "libikpso_oracle_fma.so"
    src = [str(ROOT / "oracle" / "ikpso_oracle.c"), str(ROOT / "oracle" / "ikpso_gjk.c")]
    r = subprocess.run(["gcc", "-O2", "-std=c11", "-march=native", "-mfma", "-ffp-contract=fast", "-fopenmp",
                        "-fPIC", "-shared", *src, "-o", str(out), "-lm"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip(f"no FMA build on this host: {r.stderr[-200:]}")
    return oracle._bind(ctypes.CDLL(str(out)))


def _pair(oracle, fma, chain, tg, P, I, **kw):
    B = tg.shape[0]
    a1, f1, _ = oracle.solve_batch(chain, tg, None, P, I, oracle.init_generators(B * P, 0), threads=8, **kw)
    a2, f2, _ = oracle.solve_batch(chain, tg, None, P, I, oracle.init_generators(B * P, 0), threads=8, lib=fma,
                                   **kw)
    return np.max(np.abs(a1 - a2)), np.max(np.abs(f1 - f2) / f1)


def test_reference_scene_tier_a_window(oracle, fma_oracle):
    wl = ikpso.workload(3)
    dth, dfit = _pair(oracle, fma_oracle, wl.chain, wl.targets(0, 8), 512, 20)
    assert dth < 1e-6 and dfit < 1e-6


def test_dh_arm_tier_a_window(oracle, fma_oracle):
    arm = dh_arm(IIWA["a"], IIWA["alpha"], IIWA["d"], -LIM, LIM)
    chain, mask = arm.origin.to_cuda(), arm.axis_mask
    rng = np.random.default_rng(5)
    th = rng.uniform(-0.8, 0.8, (8, 7)) * LIM
    tg = np.array([dh_forward(t, IIWA["d"], IIWA["a"], IIWA["alpha"]) for t in th], np.float32).reshape(8, 1, 3)
    d10, f10 = _pair(oracle, fma_oracle, chain, tg, 1024, 10, axis_mask=mask)
    d20, f20 = _pair(oracle, fma_oracle, chain, tg, 1024, 20, axis_mask=mask)
    assert d10 < 1e-5 and f10 < 1e-6
    assert f20 < 1e-5           # the fitness still agrees at I = 20 ...
    assert d20 > 10 * d10       # ... while the angles have started to drift apart
