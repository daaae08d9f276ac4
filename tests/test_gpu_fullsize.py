"""BASELINE configs 4 and 5 at their full sizes on one GPU, through
size-independent properties (the oracle cannot run them in test time):

  * shard invariance: the batch split the way bench.py / torchrun split it over
    8 ranks (config 4: 8 x 8192 swarms; config 5: 8 x 1024) gives per-swarm
    results bit-identical to one launch over the whole batch (global seeds);
  * the reported residual is the residual of the reported angles (oracle
    `checkDistance` restatement on a sample of swarms);
  * the reported fitness is the fitness of the reported angles (oracle
    restatement of calculateDistance on the sample, config 5's soft
    joint-limit penalty included; FAST tolerance 1e-5);
  * answers are finite and inside the joint limits.
"""
import numpy as np
import pytest

import ikpso

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def solve(wl, first, count, **kw):
    s = ikpso.BatchSolver(wl.chain, wl.particles, pso=wl.pso, limit_weight=wl.limit_weight, soft_lo=wl.soft_lo,
                          soft_hi=wl.soft_hi, **kw)
    s.seed(count, first_swarm=first)
    tg = torch.from_numpy(wl.targets(first, count)).cuda()
    out = [t.cpu().numpy() for t in s.solve(tg, iterations=wl.iterations)]
    kernel = s.kernel
    s.close()
    return out, kernel


@pytest.mark.parametrize("config,world", [(4, 8), (5, 8)])
def test_fullsize_shards_match_one_launch(oracle, device, config, world):
    wl = ikpso.workload(config)
    total = wl.swarms
    (ang, fit, res), kernel = solve(wl, 0, total)
    assert ("resident" if config == 4 else "coop") in kernel
    per = total // world
    for r in range(world):
        (a, f, q), _ = solve(wl, r * per, per)
        sl = slice(r * per, (r + 1) * per)
        assert np.array_equal(a, ang[sl]) and np.array_equal(f, fit[sl]) and np.array_equal(q, res[sl]), r

    assert np.isfinite(ang).all() and np.isfinite(fit).all() and np.isfinite(res).all()
    lo = wl.chain["min_rotation"][1:].reshape(-1)
    hi = wl.chain["max_rotation"][1:].reshape(-1)
    assert np.all(ang >= lo) and np.all(ang <= hi)  # the clamp is exact

    rng = np.random.default_rng(config)
    sample = rng.choice(total, 32, replace=False)
    tg = wl.targets(0, total)
    eff = np.flatnonzero(wl.chain["node_type"] == ikpso.NODE_EFFECTOR)  # effectors in node order
    for b in sample:
        ch = wl.chain.copy()
        ch["target_position"][eff] = tg[b]  # the swarm's own targets
        r = oracle.residual(ch, ang[b])
        assert abs(float(r) - float(res[b])) <= 1e-4 + 1e-5 * abs(float(r)), (b, r, res[b])
        # the reported fitness, soft joint-limit penalty included (config 5)
        f = oracle.fitness(ch, ang[b], limit_weight=wl.limit_weight, soft_lo=wl.soft_lo, soft_hi=wl.soft_hi)
        assert abs(float(f) - float(fit[b])) <= 1e-5 * abs(float(f)) + 1e-6, (b, f, fit[b])
