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


@pytest.fixture(scope="session")
def report():
    """report(name, dict): with IKPSO_REPORT_DIR set, a test writes the measured
    distribution behind its assertions to <dir>/<name>.json (committed under
    profiles/ so the parity claims can be audited from the repo)."""
    import json

    out = os.environ.get("IKPSO_REPORT_DIR")

    def write(name: str, data: dict) -> None:
        print(f"[{name}] " + json.dumps(data, sort_keys=True)[:2000])
        if out:
            os.makedirs(out, exist_ok=True)
            with open(os.path.join(out, name + ".json"), "w") as f:
                json.dump(data, f, indent=1, sort_keys=True)

    return write
