"""Host-side logic: scene marshalling (src/Node.h), workloads, sharding."""
import numpy as np
import pytest

import ikpso
from ikpso import dist, workloads


def test_reference_scene_marshalling():
    s = ikpso.reference_scene(reset=True)
    c = s.origin.to_cuda()
    assert c.dtype.itemsize == 88 and c.shape == (8,)
    assert c["parent_index"].tolist() == [-1, 0, 1, 2, 3, 4, 4, 4]
    assert c["node_type"].tolist() == [ikpso.NODE_ORIGIN] + [ikpso.NODE] * 4 + [ikpso.NODE_EFFECTOR] * 3
    assert np.allclose(c["rotation"][1:5], [0, 1.57, 0])
    assert np.allclose(c["rotation"][6], [0, 0, 1.57])
    assert np.all(c["length"][1:] == 1.0)
    assert np.all(c["min_rotation"][1:] == 0.0)
    assert np.all(c["max_rotation"][1:] == np.float32(2) * np.float32(np.pi))
    assert np.array_equal(c["target_position"][5:8], ikpso.RESET_TARGETS)
    assert np.all(c["effector_weight"][5:8] == 1.0)


def test_coords_roundtrip():
    s = ikpso.reference_scene()
    x = np.arange(21, dtype=np.float32) * 0.1
    s.origin.from_coords(x)
    assert np.array_equal(s.origin.to_coords(), x)
    s.reset_arm()
    assert np.array_equal(s.origin.to_coords(), s.default_coords)


def test_fill_positions_slots():
    """CopyPositions writes node i (DFS) at slot (i+1)*4; the solver reads slot (k-1)*4."""
    s = ikpso.reference_scene()
    pos = s.origin.fill_positions()
    assert pos.shape == (36,)
    assert np.allclose(pos[4:8], [0, 0, 0, 1])           # origin at slot 1
    assert np.allclose(pos[8:11], s.elbows[0].world_position())


def test_host_fk_matches_oracle(oracle):
    s = ikpso.reference_scene()
    c = s.origin.to_cuda()
    rng = np.random.default_rng(0)
    for _ in range(20):
        x = rng.uniform(0, 2 * np.pi, 21).astype(np.float32)
        s.origin.from_coords(x)
        host = np.array([n.world_position() for n in list(s.origin.dfs())[1:]])
        assert np.max(np.abs(host - oracle.node_positions(c, x))) < 2e-5


def test_splitmix64_reference_vector():
    # published splitmix64 outputs for seed 1234567
    out = workloads.splitmix64_stream(np.array([1234567], dtype=np.uint64), 5)[0].tolist()
    assert out == [6457827717110365317, 3203168211198807973, 9817491932198370423, 4593380528125082431,
                   16408922859458223821]


def test_batch_targets_deterministic_and_sharded():
    t = workloads.batch_targets(0, 64)
    assert t.shape == (64, 3, 3) and t.dtype == np.float32
    assert np.all(np.abs(t - ikpso.RESET_TARGETS[None]) <= 0.25)
    assert np.array_equal(workloads.batch_targets(10, 5), t[10:15])


def test_workloads():
    for n in (1, 2, 3, 4):
        wl = ikpso.workload(n)
        assert wl.dof == 21 and wl.chain.shape == (8,)
    w5 = ikpso.workload(5)
    assert w5.dof == 60 and w5.particles == 4096 and w5.limit_weight == 10.0
    assert w5.chain["node_type"].tolist().count(ikpso.NODE_EFFECTOR) == 1
    t = w5.targets(0, 100)
    r = np.linalg.norm(t[:, 0], axis=1)
    assert np.all(r >= 2.0) and np.all(r <= 4.0 + 1e-5)


@pytest.mark.parametrize("total,world", [(10, 3), (65536, 8), (5, 8), (0, 2), (4096, 1)])
def test_shard_range(total, world):
    ranges = [dist.shard_range(total, world, r) for r in range(world)]
    assert sum(c for _, c in ranges) == total
    nxt = 0
    for f, c in ranges:
        assert f == nxt
        nxt = f + c
    assert max(c for _, c in ranges) - min(c for _, c in ranges) <= 1
