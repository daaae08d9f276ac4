"""Cooperative resident kernel (csrc/ikpso_coop.h): one swarm over G
co-resident workgroups exchanging chunk minima through L2 every iteration.
Same algorithm and draw order as the reference, so REFERENCE arithmetic is
compared with the oracle bit for bit, including swarms that are not a
multiple of the workgroup size and groups that solve several swarms in turn."""
import numpy as np
import pytest

import ikpso

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


@pytest.mark.parametrize("P,I", [(2048, 20), (3000, 7)])
def test_coop_compat_reference_bitexact(oracle, device, monkeypatch, P, I):
    chain = ikpso.reference_scene(reset=True).origin.to_cuda()
    monkeypatch.setenv("IKPSO_ARITH", "reference")
    monkeypatch.setenv("IKPSO_KERNEL", "coop")
    D = 21
    parts = ikpso.particles_tensor(P, D)
    bests = torch.zeros(P, dtype=torch.float32, device="cuda")
    r = ikpso.rng_tensor(P)
    assert ikpso.init_generators(r, P) == 0
    res = np.zeros(D, dtype=np.float32)
    assert ikpso.calculate_pso(parts, None, bests, r, P, chain, ikpso.PSOConfig(0.5, 0.5, 1.25, I),
                               ikpso.MAIN_FITNESS, res) == 0
    ostate = oracle.init_generators(P, 0)
    ores, oparts, obests = oracle.calculate_pso(chain, P, ostate, iterations=I)
    assert np.array_equal(r.cpu().numpy()[:, :6], ostate.view(np.int32).reshape(P, 12)[:, :6])
    assert np.array_equal(bests.cpu().numpy(), obests)
    assert np.array_equal(parts.cpu().numpy(), oparts)
    assert np.array_equal(res, ores)


def test_coop_batch_groups_loop_over_swarms(oracle, device):
    """P = 16384 (G = 16 workgroups per swarm, at most 16 concurrent groups on 256
    CUs): 20 swarms, so some groups solve two swarms back to back."""
    wl = ikpso.workload(3)
    B, P, I = 20, 16384, 4
    tg = wl.targets(0, B)
    s = ikpso.BatchSolver(wl.chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith="reference", kernel="coop")
    assert "coop" in s.kernel
    s.seed(B)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    s.close()
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, ores = oracle.solve_batch(wl.chain, tg, None, P, I, ostate, threads=8)
    assert np.array_equal(ang, oang) and np.array_equal(fit, ofit)
    assert np.max(np.abs(res - ores)) < 1e-5


def test_coop_equals_streaming(device):
    """FAST: the two multi-workgroup families agree to the FAST tolerance; their
    generator streams (integer work) are identical."""
    wl = ikpso.workload(3)
    B, P, I = 16, 4096, 30
    tg = wl.targets(0, B)
    out = []
    for kern in ("coop", "streaming"):
        s = ikpso.BatchSolver(wl.chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), kernel=kern)
        s.seed(B)
        out.append([t.cpu().numpy() for t in s.solve(dev(tg), iterations=I)])
        s.close()
    (a1, f1, r1), (a2, f2, r2) = out
    assert np.all(np.isfinite(f1))
    assert np.mean(np.abs(f1 - f2) / f2 <= 1e-3) >= 0.75
    assert abs(f1.mean() - f2.mean()) / f2.mean() < 5e-3


def test_coop_visualiser_swarm_auto(oracle, device, monkeypatch):
    """AUTO picks the cooperative kernel for the visualiser's N = 16384; a few
    such swarms run the latency variant with generator waves, each swarm's 64
    chunks a group wider than an XCD (linear membership, cross-XCD hand-offs):
    REFERENCE bit-exact to the oracle, and a full batch goes back to the
    throughput plan."""
    chain = ikpso.reference_scene(reset=True).origin.to_cuda()
    B, P, I = 2, 16384, 5
    s = ikpso.BatchSolver(chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith="reference")
    assert "coop" in s.kernel
    tg = ikpso.workload(3).targets(0, B)
    s.seed(8)
    ang, fit, res = (t.cpu().numpy() for t in s.solve(dev(tg), iterations=I))
    assert s.kernel == "swarm_coop<ref_tree7> (latency variant, generator waves)", s.kernel
    states = s.generator_states(0, B)
    s.solve(dev(ikpso.workload(3).targets(0, 8)), iterations=1)
    assert s.kernel == "swarm_coop<ref_tree7>", s.kernel
    s.close()
    ostate = oracle.init_generators(B * P, 0)
    oang, ofit, ores = oracle.solve_batch(chain, tg, None, P, I, ostate, threads=8)
    assert np.array_equal(ang, oang) and np.array_equal(fit, ofit)
    assert np.array_equal(states[:, :6], ostate.view(np.int32).reshape(B * P, 12)[:, :6])


def test_auto_reports_latency_variant(device):
    """AUTO routes a few swarms to the cooperative latency variant and a full
    batch to the resident kernel; the solver's kernel name follows each call."""
    wl = ikpso.workload(3)
    s = ikpso.BatchSolver(wl.chain, 1024, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, 5))
    assert s.kernel == "swarm_resident<ref_tree7>"
    s.seed(512)
    s.solve(dev(wl.targets(0, 1)), iterations=5)
    assert s.kernel == "swarm_coop<ref_tree7> (latency variant, generator waves)"
    s.solve(dev(wl.targets(0, 512)), iterations=5)
    assert s.kernel == "swarm_resident<ref_tree7>"
    s.close()


# ------------------------------------------------- contention fallback
# IKPSO_COOP_SPIN_LIMIT=0 makes every group wait give up at its first unmet poll:
# the path a solve takes when other work on the GPU keeps a group from
# assembling.  The solve must still complete -- restored generator states,
# re-run on the streaming kernels -- with the results a streaming solve gives.

@pytest.mark.parametrize("B", [1, 6])
def test_coop_forced_timeout_falls_back_batch(device, monkeypatch, B):
    """B = 6: the snapshot is a copy before the launch; B = 1: the kernel writes
    it as its chunks load the states.  Then two more solves on the same solvers
    (the slots re-cleared after the fallback's streaming pass, then numbered
    past the last solve's tags) still equal the streaming solver's."""
    wl = ikpso.workload(3)
    P, I = 16384, 5
    tg = dev(wl.targets(0, B))
    out = {}
    for name, kern, spin in (("coop", "coop", "0"), ("streaming", "streaming", None)):
        if spin is None:
            monkeypatch.delenv("IKPSO_COOP_SPIN_LIMIT", raising=False)
        else:
            monkeypatch.setenv("IKPSO_COOP_SPIN_LIMIT", spin)
        s = ikpso.BatchSolver(wl.chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), arith="reference", kernel=kern)
        s.seed(B)
        # without sync the aborted groups' swarms read as NaN ...
        a0, f0, r0 = s.solve(tg, iterations=I, sync=False)
        if kern == "coop":
            torch.cuda.synchronize()
            assert torch.isnan(f0).any() and torch.isnan(a0).any()
            before = s.fallbacks
            s.sync()  # ... and sync re-runs the batch from the snapshot
            assert s.fallbacks == before + 1
            monkeypatch.delenv("IKPSO_COOP_SPIN_LIMIT", raising=False)
        res = [t.cpu().numpy() for t in (a0, f0, r0)]
        for _ in range(2):
            res += [t.cpu().numpy() for t in s.solve(tg, iterations=I)]
        if kern == "coop":
            assert s.fallbacks == before + 1
        out[name] = res
        s.close()
    for x, y in zip(out["coop"], out["streaming"]):
        assert np.array_equal(x, y)


def test_coop_forced_timeout_falls_back_compat(oracle, device, monkeypatch):
    """calculatePSO (the visualiser's N = 16384, cooperative by AUTO) returns
    success and the oracle's bit-exact state even when every group gives up."""
    monkeypatch.setenv("IKPSO_ARITH", "reference")
    monkeypatch.setenv("IKPSO_COOP_SPIN_LIMIT", "0")
    lib = ikpso.load()
    chain = ikpso.reference_scene(reset=True).origin.to_cuda()
    P, I, D = 16384, 3, 21
    parts = ikpso.particles_tensor(P, D)
    bests = torch.zeros(P, dtype=torch.float32, device="cuda")
    r = ikpso.rng_tensor(P)
    assert ikpso.init_generators(r, P) == 0
    res = np.zeros(D, dtype=np.float32)
    before = lib.ikpso_coop_fallbacks()
    assert ikpso.calculate_pso(parts, None, bests, r, P, chain, ikpso.PSOConfig(0.5, 0.5, 1.25, I),
                               ikpso.MAIN_FITNESS, res) == 0
    assert lib.ikpso_coop_fallbacks() == before + 1
    ostate = oracle.init_generators(P, 0)
    ores, oparts, obests = oracle.calculate_pso(chain, P, ostate, iterations=I)
    assert np.array_equal(r.cpu().numpy()[:, :6], ostate.view(np.int32).reshape(P, 12)[:, :6])
    assert np.array_equal(bests.cpu().numpy(), obests)
    assert np.array_equal(parts.cpu().numpy(), oparts)
    assert np.array_equal(res, ores)


def test_compat_frames_across_families_and_fallback(oracle, device, monkeypatch):
    """The per-frame call keeps its aux block, its cooperative slots (exchanges
    numbered past the last frame's tags instead of cleared) and its generator
    snapshot (written by the kernel) between frames.  A sequence that changes
    what lies in the scratch under it -- streaming frames over the slots, a
    forced fallback, another swarm size, new distance-term positions, the answer
    into device memory -- stays the oracle's bit for bit, frame after frame."""
    monkeypatch.setenv("IKPSO_ARITH", "reference")
    monkeypatch.delenv("IKPSO_COOP_SPIN_LIMIT", raising=False)
    monkeypatch.delenv("IKPSO_KERNEL", raising=False)
    lib = ikpso.load()
    scene = ikpso.reference_scene(reset=True)
    D, I = 21, 3
    streams = {}
    for n in (16384, 512):
        r = ikpso.rng_tensor(n)
        assert ikpso.init_generators(r, n) == 0
        streams[n] = (r, oracle.init_generators(n, 0), ikpso.particles_tensor(n, D),
                      torch.zeros(n, dtype=torch.float32, device="cuda"))
    pos0 = scene.origin.fill_positions()
    steps = [dict(), dict(kernel="streaming"), dict(), dict(spin="0"), dict(), dict(device_result=True),
             dict(n=512), dict(), dict(positions=pos0), dict(positions=pos0 + 0.25), dict(), dict()]
    pose = None
    for k, stp in enumerate(steps):
        n = stp.get("n", 16384)
        r, ost, parts, bests = streams[n]
        for var, val in (("IKPSO_KERNEL", stp.get("kernel")), ("IKPSO_COOP_SPIN_LIMIT", stp.get("spin"))):
            if val is None:
                monkeypatch.delenv(var, raising=False)
            else:
                monkeypatch.setenv(var, val)
        if pose is not None:
            scene.origin.from_coords(pose)
        chain = scene.origin.to_cuda()
        pos = stp.get("positions")
        fit = ikpso.FitnessConfig(3.0, 1.0 if pos is not None else 0.0, 0.1)
        res = torch.zeros(D, dtype=torch.float32, device="cuda") if stp.get("device_result") else \
            np.zeros(D, dtype=np.float32)
        before = lib.ikpso_coop_fallbacks()
        assert ikpso.calculate_pso(parts, pos, bests, r, n, chain, ikpso.PSOConfig(0.5, 0.5, 1.25, I), fit, res) == 0
        assert lib.ikpso_coop_fallbacks() == before + (1 if stp.get("spin") == "0" else 0), k
        ores, oparts, obests = oracle.calculate_pso(chain, n, ost, iterations=I, distance_weight=fit.distance_weight,
                                                    positions=pos)
        got = res.cpu().numpy() if isinstance(res, torch.Tensor) else res
        assert np.array_equal(got, ores), (k, stp)
        assert np.array_equal(bests.cpu().numpy(), obests), (k, stp)
        assert np.array_equal(r.cpu().numpy()[:, :6], ost.view(np.int32).reshape(n, 12)[:, :6]), (k, stp)
        if n == 16384:
            pose = got.copy()


def test_solve_rejects_wrong_dtype_and_device(device):
    wl = ikpso.workload(3)
    s = ikpso.BatchSolver(wl.chain, 64)
    s.seed(2)
    tg = dev(wl.targets(0, 2))
    with pytest.raises(ValueError):
        s.solve(tg.double(), iterations=1)
    with pytest.raises(ValueError):
        s.solve(tg.cpu(), iterations=1)
    with pytest.raises(ValueError):
        s.evaluate(torch.zeros((3, 21), dtype=torch.float64, device="cuda"))
    s.close()
