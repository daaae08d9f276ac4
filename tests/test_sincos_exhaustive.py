"""REFERENCE arithmetic's sin/cos (ikpso_device.h:sincos_reference) against the
CPU oracle's (float)sin((double)x) / (float)cos((double)x) on EVERY float with
|x| < 4096 -- 2.33e9 arguments, both signs, zeros and subnormals -- bit for bit.

The reference's FK calls precise sinf/cosf on every joint angle
(rotateMatrixAlong{X,Y,Z}, src/matrix_operations.cuh:123-161); the oracle restates
them as correctly rounded fp32 of the fp64 libm value, and the REFERENCE kernels'
bit-identity with the oracle (tests/test_gpu_parity.py, the 731-call recorded
trajectory) rests on this routine agreeing on every argument the kernels can
meet.  An exhaustive check needs no runtime rounding test: the routine is
legitimate iff it reports zero mismatches here.  The same routine compiled for
the host (explicit fma builtins, no contraction) as the device uses.
~25 s on 8 host threads."""
import json
import os
import subprocess
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "inverse-kinematics-pso-research_amd" / "csrc"


def run_exhaustive(fast: bool = False) -> dict:
    with tempfile.TemporaryDirectory() as td:
        exe = Path(td) / "sincos_exhaustive"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", f"-I{CSRC}",
                        f"-I{ROOT / 'include'}", str(ROOT / "tests" / "sincos_exhaustive.cpp"), "-o", str(exe)],
                       check=True, capture_output=True)
        threads = len(os.sched_getaffinity(0))
        out = subprocess.run([str(exe), str(threads), "1" if fast else "0"], capture_output=True, text=True,
                             check=True, timeout=1800).stdout
    return json.loads(out.strip().splitlines()[-1])


def test_reference_sincos_every_float():
    r = run_exhaustive()
    assert r["floats"] == 2 * 0x45800000
    assert r["reference_sin_mismatch"] == 0 and r["reference_cos_mismatch"] == 0, r
