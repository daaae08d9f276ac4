"""Source hash of the HIP library (``ikpso_build_id()`` in include/ikpso.h).

The Makefile compiles this hash into libikpso.so; the loader (``_abi.load``)
recomputes it from the tree it runs from and refuses a library built from other
sources -- a failed rebuild can no longer leave an older library in place to be
measured or tested as if it were the current one.  Stdlib only: the Makefile
runs it as a script.

    python3 _buildid.py [EXTRA]   prints the id; a variant build's extra compiler
                                  flags append "+" and their hash
"""
from __future__ import annotations

import hashlib
import sys
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parents[1]  # inverse-kinematics-pso-research_amd
ROOT = PKG_ROOT.parent


def source_files():
    """The library's sources: csrc/*.{h,hip,cpp}, csrc/Makefile, include/*.h."""
    csrc = PKG_ROOT / "csrc"
    files = [p for p in csrc.iterdir() if p.is_file() and (p.suffix in (".h", ".hip", ".cpp") or p.name == "Makefile")]
    files += [p for p in (ROOT / "include").iterdir() if p.is_file() and p.suffix == ".h"]
    return sorted(files, key=lambda p: p.relative_to(ROOT).as_posix())


def tree_id() -> str | None:
    """16 hex digits over (path, bytes) of every source file; None without sources."""
    try:
        files = source_files()
    except OSError:
        return None
    if not files:
        return None
    h = hashlib.sha256()
    for p in files:
        h.update(p.relative_to(ROOT).as_posix().encode())
        h.update(b"\0")
        h.update(p.read_bytes())
        h.update(b"\0")
    return h.hexdigest()[:16]


def build_id(extra: str = "") -> str:
    tid = tree_id() or "unknown"
    extra = " ".join(extra.split())
    return tid if not extra else f"{tid}+{hashlib.sha256(extra.encode()).hexdigest()[:8]}"


if __name__ == "__main__":
    print(build_id(sys.argv[1] if len(sys.argv) > 1 else ""))
