"""The caller-side examples (examples/): the reference visualiser's frame loop
linked through the reference's own C++ entry points (compat_frames.cpp), and the
batched C ABI from plain C (batch_c.c) -- no Python on the product side."""
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EX = Path(__file__).resolve().parents[1] / "examples" / "_build"


def run(*args, timeout=120):
    exe = EX / args[0]
    if not exe.exists():
        pytest.fail(f"{exe} not built (__graft_entry__.build() builds examples/)")
    return subprocess.run([str(exe), *map(str, args[1:])], capture_output=True, text=True, timeout=timeout)


def test_compat_visualiser_loop(device):
    r = run("compat_frames", 3, 16384)
    assert r.returncode == 0, r.stdout + r.stderr
    frames = [int(x) for x in re.search(r"frames to converge:(.*)", r.stdout).group(1).split()]
    assert len(frames) == 3 and all(3 <= f < 2000 for f in frames), r.stdout


def test_batch_from_plain_c(device):
    r = run("batch_c", 64, 100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "finite 1" in r.stdout and "particle-updates/s" in r.stdout, r.stdout


@pytest.mark.parametrize("arith", ["reference", "fast"])
def test_compat_entry_replays_recorded_frames(golden, arith):
    """The visualiser's exact call shape through the mangled calculatePSO
    (src/Main.cpp:28-29,145,225): 70 unrecorded frames, then R and frames 70-74
    with the answer fed back, against results.xlsx DEGREES_3 rows 3-7 (see
    tests/test_trajectory.py).  REFERENCE: bit-identical to the oracle's replay
    and within 1e-5 rad of the reference's own log; FAST: within 1e-4."""
    import os

    with np.load(golden / "trajectory3.npz", allow_pickle=False) as z:
        log, orc, k0 = z["degrees"][1:6], z["oracle_chained"], int(z["meta"][4])
    env = dict(os.environ, IKPSO_ARITH=arith)
    exe = EX / "compat_frames"
    if not exe.exists():
        pytest.fail(f"{exe} not built (__graft_entry__.build() builds examples/)")
    r = subprocess.run([str(exe), "replay", str(k0), "5", "16384"], capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("frame ")]
    assert [int(ln.split(":")[0].split()[1]) for ln in lines] == list(range(k0, k0 + 5))
    got = np.array([[float(x) for x in ln.split(":")[1].split()] for ln in lines], dtype=np.float32)
    if arith == "reference":
        assert np.array_equal(got, orc)
        assert np.max(np.abs(got - log)) <= 1e-5
    else:
        assert np.max(np.abs(got - log)) <= 1e-4, np.max(np.abs(got - log), axis=1)
