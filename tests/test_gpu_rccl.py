"""The RCCL branch of the multi-GPU path, executed on the one lease GPU.

bench.py's N > 1 ranks initialise a "nccl" (= RCCL) process group with
device_id and all-gather the per-swarm result rows once per step
(ikpso/dist.py: gather_rows -> all_gather_into_tensor).  The round's 8-GPU run
is the driver's; this makes sure that branch has executed on hardware before:
a world-1 RCCL group on cuda:0, gather_rows forced through the collective.
"""
import socket

import numpy as np
import pytest

import ikpso
from ikpso import dist as idist

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture()
def rccl_world1(device):
    import torch.distributed as dist

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        yield dist
    finally:
        dist.destroy_process_group()


def test_rccl_gather_rows_world1(rccl_world1):
    rows = torch.randn(37, 23, device="cuda")
    out = idist.gather_rows(rows, 37, 1, force=True)
    torch.cuda.synchronize()
    assert out.device == rows.device and torch.equal(out, rows)


def test_rccl_gathers_solver_results(rccl_world1):
    """bench.py's step on one rank: solve, pack, all-gather over RCCL, copy to host."""
    wl = ikpso.workload(3)
    B, P, I = 16, 1024, 10
    s = ikpso.BatchSolver(wl.chain, P, pso=wl.pso)
    s.seed(B)
    ang, fit, res = s.solve(torch.from_numpy(wl.targets(0, B)).cuda(), iterations=I)
    rows = idist.pack_results(ang, fit, res)
    got = idist.gather_rows(rows, B, 1, force=True).cpu().numpy()
    s.close()
    want = np.concatenate([ang.cpu().numpy(), fit.cpu().numpy()[:, None], res.cpu().numpy()[:, None]], axis=1)
    assert np.array_equal(got, want)
    rccl_world1.barrier()
