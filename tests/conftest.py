import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG_ROOT = ROOT / "inverse-kinematics-pso-research_amd"
GOLDEN = Path(__file__).resolve().parent / "golden"
for p in (ROOT, PKG_ROOT, ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc  # tests/ may use the oracle as the checker

    orc.load()
    return orc


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


@pytest.fixture(scope="session")
def fk_kat():
    with np.load(GOLDEN / "fk_kat.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def distance_kat():
    with np.load(GOLDEN / "distance_kat.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
