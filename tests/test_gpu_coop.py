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

def test_coop_forced_timeout_falls_back_batch(device, monkeypatch):
    wl = ikpso.workload(3)
    B, P, I = 6, 16384, 5
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
        out[name] = [t.cpu().numpy() for t in (a0, f0, r0)]
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
