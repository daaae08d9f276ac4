"""The oracle pinned against the reference's own recorded CUDA run.

Documentation/results.xlsx DEGREES_3 is one consecutive recording of the
visualiser (src/Main.cpp:163-227): 662 rows = sum FRAMES_3, one calculatePSO
per frame (N = 16384, 15 iterations, src/Main.cpp:17,130), the generator states
carried across frames from one initGenerators (:145).  Every call draws exactly
D + 3*D*I = 966 uniforms per particle whatever the pose, so the solve logged in
row r ran on the initGenerators states advanced by (r + 67) * 966 draws (row 3
is frame 70).  tests/golden/make_golden.py (make_trajectory) documents the
row/frame/case map and wrote tests/golden/trajectory3.npz.

What this pins against the real reference run (tolerance 1e-5 rad: the log has
6 significant digits, the reference ran nvcc's FMA contraction and CUDA's
sinf/cosf): cuRAND's seeding constants and uniform mapping, the r1/r2/r3 draw
order, the update, the clamp, the FK, the fitness and the 16384-particle
first-minimum argmin.  The GPU side is tests/test_gpu_trajectory.py.
"""
import numpy as np
import pytest

import ikpso


@pytest.fixture(scope="module")
def traj(golden):
    with np.load(golden / "trajectory3.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def meta(t):
    N, I, D, draws, k0 = (int(x) for x in t["meta"])
    return N, I, D, draws, k0


def test_fixture_is_one_recording(traj):
    """Row/frame/case bookkeeping: contiguous rows, frames = rows + 67, cases of
    FRAMES_3's lengths, exactly one converged row (checkDistance <= 0.025 on
    the logged effector positions) per case, and it is the case's last."""
    N, I, D, draws, k0 = meta(traj)
    assert (N, I, D, draws, k0) == (16384, 15, 21, 21 + 3 * 21 * 15, 70)
    rows, frame, case = traj["rows"], traj["frame"], traj["case"]
    assert rows.tolist() == list(range(2, 2 + int(traj["frames"].sum())))
    assert np.array_equal(frame, rows + 67)
    assert np.bincount(case)[1:].tolist() == traj["frames"].tolist()
    eff = traj["positions"][:, 12:21].reshape(-1, 3, 3)
    dist = np.linalg.norm(eff - ikpso.scene.RESET_TARGETS[None].astype(np.float64), axis=2).sum(axis=1)
    last = np.r_[case[1:] != case[:-1], True]
    assert np.all(dist[last] <= 0.025 + 1e-5)
    assert np.all(dist[~last & ~traj["stale"]] > 0.025 - 1e-5)
    starts = np.flatnonzero(traj["from_default"])
    assert len(starts) == 20 and rows[starts[0]] == 3


def test_skipahead_equals_stepping(oracle):
    a = oracle.init_generators(16, 1000)
    b = a.copy()
    oracle.skipahead(a, 966 * 3 + 5)
    for i in range(16):
        oracle.raw_stream(b[i:i + 1], 966 * 3 + 5)
    assert a.tobytes() == b.tobytes()


def replay(oracle, traj, frame, pose):
    N, I, D, draws, _ = meta(traj)
    scene = ikpso.reference_scene(reset=True)
    if pose is not None:
        scene.origin.from_coords(np.asarray(pose, dtype=np.float32))
    st = oracle.init_generators(N, 0)
    oracle.skipahead(st, frame * draws)
    res, _, _ = oracle.calculate_pso(scene.origin.to_cuda(), N, st, iterations=I,
                                     positions=scene.origin.fill_positions())
    return res


def test_oracle_reproduces_recorded_frames_70_to_74(oracle, traj):
    """Frames 70-74 (rows 3-7) from the default pose with the oracle's own answer
    fed back, as the visualiser does: within 1e-5 of the log on every angle."""
    pose = None
    for r in range(3, 8):
        i = r - 2
        res = replay(oracle, traj, int(traj["frame"][i]), pose)
        assert np.array_equal(res, traj["oracle_chained"][r - 3]), r
        assert np.max(np.abs(res - traj["degrees"][i])) <= 1e-5, (r, np.max(np.abs(res - traj["degrees"][i])))
        pose = res


@pytest.mark.parametrize("case", [2, 20])
def test_oracle_reproduces_case_starts(oracle, traj, case):
    """The first solve of a case (from the default pose after resetArm) hundreds of
    frames into the recording: within 1e-5 of the log."""
    i = int(np.flatnonzero(traj["from_default"] & (traj["case"] == case))[0])
    res = replay(oracle, traj, int(traj["frame"][i]), None)
    assert np.array_equal(res, traj["oracle_step"][i])
    assert np.max(np.abs(res - traj["degrees"][i])) <= 1e-5


def test_one_step_replay_envelope(traj):
    """The committed one-step replay (each frame from the previous row's logged
    pose, generator states at its frame): every case start and >= 75 % of all
    rows within 1e-5 of the log; the rest are argmin switches (>= 1e-4) that
    the 6-digit start pose or the reference's FMA/sinf rounding decide.  The
    two populations do not overlap much, which is what makes the 1e-5 bound a
    pin rather than a fit (stated in DESIGN.md §3)."""
    ok = ~traj["stale"]
    err = traj["oracle_step_err"][ok]
    assert np.all(traj["oracle_step_err"][traj["from_default"]] <= 1e-5)
    assert np.mean(err <= 1e-5) >= 0.75, np.mean(err <= 1e-5)
    assert np.sum((err > 1e-5) & (err < 1e-4)) <= 5


def test_one_step_sample_recomputes(oracle, traj):
    """Two committed one-step rows (one on each side of the envelope) are what the
    oracle computes now."""
    ok = np.flatnonzero(~traj["stale"] & ~traj["from_default"])
    near = ok[traj["oracle_step_err"][ok] <= 1e-5][10]
    far = ok[traj["oracle_step_err"][ok] > 1e-4][0]
    for i in (near, far):
        res = replay(oracle, traj, int(traj["frame"][i]), traj["degrees"][i - 1])
        assert np.array_equal(res, traj["oracle_step"][i]), int(traj["rows"][i])


def test_unpinned_rows_are_near_ties(oracle, traj):
    """The rows the one-step replay does not reproduce to 1e-5 (155 of 661) are
    another particle of (nearly) the same fitness winning: the reference's
    logged answer and the replay's score alike under the frame's own fitness
    (the previous row's pose as the angle term's rest pose, the reset targets) --
    median |df|/f 4e-5, 91 % within 1e-3, worst 1.1e-2, and the log is better
    about as often as the replay -- and their residuals agree to 1.6e-3."""
    ok = ~traj["stale"]
    rows = np.flatnonzero(ok & (traj["oracle_step_err"] > 1e-5))
    rel, dres = [], []
    for i in rows:
        scene = ikpso.reference_scene(reset=True)
        if not traj["from_default"][i]:
            scene.origin.from_coords(traj["degrees"][i - 1].astype(np.float32))
        chain = scene.origin.to_cuda()
        logged = traj["degrees"][i].astype(np.float32)
        f_log, f_rep = oracle.fitness(chain, logged), oracle.fitness(chain, traj["oracle_step"][i])
        rel.append((float(f_log) - float(f_rep)) / float(f_rep))
        dres.append(float(oracle.residual(chain, logged)) - float(oracle.residual(chain, traj["oracle_step"][i])))
    rel, dres = np.array(rel), np.array(dres)
    assert len(rows) < 0.25 * ok.sum()
    assert np.median(np.abs(rel)) < 1e-4 and np.mean(np.abs(rel) < 1e-3) > 0.85 and np.abs(rel).max() < 2e-2
    assert 0.25 < np.mean(rel > 0) < 0.75  # neither side systematically better
    assert np.abs(dres).max() < 5e-3
