"""The caller-side examples (examples/): the reference visualiser's frame loop
linked through the reference's own C++ entry points (compat_frames.cpp), and the
batched C ABI from plain C (batch_c.c) -- no Python on the product side."""
import re
import subprocess
from pathlib import Path

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
