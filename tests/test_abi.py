"""The C-ABI library: loads, exports every declared symbol, struct layouts,
argument validation that returns before any device work."""
import ctypes
import re
import subprocess
import tempfile
from pathlib import Path

import numpy as np
import pytest

import ikpso
from ikpso import _abi

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "ikpso.h"


def declared_symbols():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ikpso_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = _abi.load()
    names = declared_symbols()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_abi.SIGNATURES), "python signatures out of sync with include/ikpso.h"
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_abi.LIB_PATH)], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}$", nm, re.M), n


def test_compat_symbols_exported():
    """The reference's own (C++-mangled) entry points for a drop-in link."""
    nm = subprocess.run(["nm", "-DC", "--defined-only", str(_abi.LIB_PATH)], capture_output=True, text=True).stdout
    assert "initGenerators(curandStateXORWOW*, int)" in nm
    assert ("calculatePSO(float*, float*, float*, curandStateXORWOW*, int, NodeCUDA*, PSOConfig, FitnessConfig, "
            "Coordinates*, obj*, int)") in nm


def test_abi_version_and_strings():
    lib = _abi.load()
    assert lib.ikpso_abi_version() == 5
    assert lib.ikpso_status_string(0) == b"ok"
    assert lib.ikpso_status_string(2) == b"unsupported configuration"


def test_struct_layouts_match_header():
    src = r'''
    #include <stdio.h>
    #include <stddef.h>
    #include "ikpso.h"
    int main(void) {
      printf("%zu %zu %zu %zu %zu\n", sizeof(ikpso_node), sizeof(ikpso_rng_state), sizeof(ikpso_pso_config),
             sizeof(ikpso_fitness_config), sizeof(ikpso_collider));
      printf("%zu %zu %zu %zu %zu %zu %zu\n", offsetof(ikpso_node, position), offsetof(ikpso_node, rotation),
             offsetof(ikpso_node, max_rotation), offsetof(ikpso_node, min_rotation), offsetof(ikpso_node, length),
             offsetof(ikpso_node, target_position), offsetof(ikpso_collider, quat));
      printf("%zu %zu %zu %zu %zu %zu\n", sizeof(ikpso_solver_desc), offsetof(ikpso_solver_desc, positions),
             offsetof(ikpso_solver_desc, soft_hi), offsetof(ikpso_solver_desc, colliders),
             offsetof(ikpso_solver_desc, collider_count), offsetof(ikpso_solver_desc, axis_mask));
      return 0; }
    '''
    with tempfile.TemporaryDirectory() as td:
        c = Path(td) / "p.c"
        c.write_text(src)
        exe = Path(td) / "p"
        subprocess.run(["gcc", "-I", str(ROOT / "include"), str(c), "-o", str(exe)], check=True)
        out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    sizes = list(map(int, out[0].split()))
    assert sizes == [88, 48, 16, 12, 48]
    offs = list(map(int, out[1].split()))
    nd = ikpso.NODE_DTYPE
    assert offs[:6] == [nd.fields[f][1] for f in
                        ("position", "rotation", "max_rotation", "min_rotation", "length", "target_position")]
    assert offs[6] == 32  # float4 quat is 16-byte aligned in obj_t
    d = list(map(int, out[2].split()))
    assert d[0] == ctypes.sizeof(_abi.SolverDesc)
    assert d[1] == _abi.SolverDesc.positions.offset and d[2] == _abi.SolverDesc.soft_hi.offset
    assert d[3] == _abi.SolverDesc.colliders.offset and d[4] == _abi.SolverDesc.collider_count.offset
    assert d[5] == _abi.SolverDesc.axis_mask.offset
    assert _abi.COLLIDER_DTYPE.fields["quat"][1] == offs[6]


def test_validation_without_device_work():
    lib = _abi.load()
    assert lib.ikpso_solver_create(None, ctypes.byref(ctypes.c_void_p())) == _abi.IKPSO_ERR_INVALID_ARG
    assert lib.ikpso_init_generators_seeded(None, 5, 0, None) == _abi.IKPSO_ERR_INVALID_ARG
    assert lib.ikpso_solver_seed(None, 1, 0, 0, None) == _abi.IKPSO_ERR_INVALID_ARG
    assert lib.ikpso_solve_batch(None, None, None, 1, 1, None, None, None, None) == _abi.IKPSO_ERR_INVALID_ARG
    assert lib.ikpso_solver_generator_states(None, 0, 1, None, None) == _abi.IKPSO_ERR_INVALID_ARG
    # a collider count without colliders is refused before any device work
    pso = _abi.PSOConfig(0.5, 0.5, 1.25, 15)
    fit = _abi.FitnessConfig(3.0, 0.0, 0.1)
    assert lib.ikpso_calculate_pso(None, None, None, None, 16, None, 8, pso, fit, None, None, 1, None) == \
        _abi.IKPSO_ERR_INVALID_ARG
    assert lib.ikpso_calculate_pso(None, None, None, None, 16, None, 8, pso, fit, None, None, -1, None) == \
        _abi.IKPSO_ERR_INVALID_ARG
    assert lib.ikpso_calculate_pso(None, None, None, None, 0, None, 8, pso, fit, None, None, 0, None) == \
        _abi.IKPSO_ERR_INVALID_ARG


def test_build_id_is_the_tree_hash():
    """The library carries the hash of the sources it was built from (make writes it)."""
    from ikpso import _buildid

    lib = _abi.load()
    assert lib.ikpso_build_id().decode() == _buildid.tree_id()
    assert len(_buildid.tree_id()) == 16
    assert _buildid.build_id("-DX=1").startswith(_buildid.tree_id() + "+")


def test_stale_library_is_refused(monkeypatch):
    """A library built from other sources (e.g. a failed rebuild left the old one
    in place) is refused at load; IKPSO_ALLOW_STALE=1 accepts it (variant builds)."""
    from ikpso import _buildid

    monkeypatch.setattr(_abi, "_LIB", None)
    monkeypatch.setattr(_buildid, "tree_id", lambda: "0123456789abcdef")
    monkeypatch.delenv("IKPSO_ALLOW_STALE", raising=False)
    with pytest.raises(_abi.StaleLibraryError, match="0123456789abcdef"):
        _abi.load()
    monkeypatch.setattr(_abi, "_LIB", None)
    monkeypatch.setenv("IKPSO_ALLOW_STALE", "1")
    assert _abi.load().ikpso_abi_version() == _abi.ABI_VERSION


def test_product_has_no_cpu_fallback():
    """The product package never imports the oracle and fails loudly without the library."""
    pkg = ROOT / "inverse-kinematics-pso-research_amd"
    for py in list(pkg.rglob("*.py")) + list(pkg.rglob("*.cpp")) + list(pkg.rglob("*.hip")):
        assert "oracle" not in py.read_text().lower().replace("oracle/", ""), py
    code = ("import sys; sys.path.insert(0, %r); import os; os.environ['IKPSO_LIB']='/nonexistent.so';"
            "from ikpso import _abi\ntry:\n _abi.load()\nexcept FileNotFoundError:\n print('LOUD')" % str(pkg))
    out = subprocess.run(["python", "-c", code], capture_output=True, text=True)
    assert "LOUD" in out.stdout


def test_compat_refuses_other_dof(tmp_path):
    """A caller compiled with another DEGREES_OF_FREEDOM than the library gets
    hipErrorInvalidConfiguration from calculatePSO (no device work), one built
    with the library's value reaches the argument checks (hipErrorInvalidValue
    for the null buffers below)."""
    src = tmp_path / "caller.cpp"
    src.write_text(
        '#include "ikpso_compat.h"\n#include <cstdio>\n'
        "int main() {\n"
        "  PSOConfig p(0.5f, 0.5f, 1.25f, 1); FitnessConfig f;\n"
        "  hipError_t e = calculatePSO(nullptr, nullptr, nullptr, nullptr, 0, nullptr, p, f, nullptr, nullptr, 0);\n"
        '  std::printf("%d\\n", (int)e); return 0; }\n')
    lib = ROOT / "inverse-kinematics-pso-research_amd" / "ikpso" / "_lib"
    codes = {}
    for dof in (21, 24):
        exe = tmp_path / f"caller{dof}"
        subprocess.run(["/opt/rocm/bin/hipcc", f"-DDEGREES_OF_FREEDOM={dof}", "-I", str(ROOT / "include"), str(src),
                        "-o", str(exe), f"-L{lib}", "-likpso", f"-Wl,-rpath,{lib}"], check=True,
                       capture_output=True)
        codes[dof] = int(subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout)
    assert codes[21] == 1      # hipErrorInvalidValue: argument checks
    assert codes[24] == 9      # hipErrorInvalidConfiguration: D mismatch
