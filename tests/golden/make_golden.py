#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ (run in the build container,
where /root/reference exists; the GPU box only reads the committed outputs).

Sources -- data only, no reference code is executed:
  * /root/reference/Documentation/results.xlsx: the reference's own diagnostic
    logs (src/Main.cpp:147-215, writer fillPositionData :306-328), i.e. rows of
    (21 joint angles -> 21 node world coordinates) printed with 6 significant
    digits, per-frame convergence distances and frames-to-converge counts.
  * rocRAND's xorwow_engine (/opt/rocm/include/rocrand/rocrand_xorwow.h), an
    in-container implementation of the XORWOW recurrence cuRAND also uses
    (its seeding differs, so only the step is compared).

Outputs:
  fk_kat.npz        degrees [N,21], positions [N,21], sheet/row ids of kept rows,
                    and the ids of rows dropped as stale (first frame after a
                    reset keypress: angles and positions from different frames)
  distance_kat.npz  joint angles [M,21], effector positions [M,3,3] and the logged
                    distance [M] (checkDistance against the reset targets)
  frames3.json      FRAMES_3 (iteration 3 = HEAD code) frames-to-converge
  xorwow_rocrand.json  rocRAND xorwow_engine::next() outputs from given states
"""
from __future__ import annotations

import json
import re
import subprocess
import sys
import tempfile
import xml.etree.ElementTree as ET
import zipfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
XLSX = Path("/root/reference/Documentation/results.xlsx")
NS = {"m": "http://schemas.openxmlformats.org/spreadsheetml/2006/main"}
RID = "{http://schemas.openxmlformats.org/officeDocument/2006/relationships}id"


def read_sheets(path: Path) -> dict:
    z = zipfile.ZipFile(path)
    ss = ET.fromstring(z.read("xl/sharedStrings.xml"))
    strings = ["".join(t.text or "" for t in si.iter("{%s}t" % NS["m"])) for si in ss.findall("m:si", NS)]
    wb = ET.fromstring(z.read("xl/workbook.xml"))
    rels = {r.get("Id"): r.get("Target") for r in ET.fromstring(z.read("xl/_rels/workbook.xml.rels"))}
    out = {}
    for s in wb.find("m:sheets", NS):
        root = ET.fromstring(z.read("xl/" + rels[s.get(RID)]))
        rows = {}
        for row in root.iter("{%s}row" % NS["m"]):
            cells = {}
            for c in row.findall("m:c", NS):
                col = re.match(r"[A-Z]+", c.get("r")).group()
                v = c.find("m:v", NS)
                if v is None:
                    continue
                val = strings[int(v.text)] if c.get("t") == "s" else v.text
                cells[col] = val
            rows[int(row.get("r"))] = cells
        out[s.get("name")] = rows
    return out


def col_name(i: int) -> str:
    return chr(ord("A") + i)


def numeric_rows(rows: dict, ncols: int) -> dict:
    """row number -> float64 vector of the first ncols columns, for fully numeric rows."""
    res = {}
    for r, cells in rows.items():
        try:
            vals = [float(cells[col_name(i)]) for i in range(ncols)]
        except (KeyError, ValueError):
            continue
        res[r] = np.array(vals)
    return res


PARENTS = [-1, 0, 1, 2, 3, 4, 4, 4]  # DFS parent indices of the reference scene (src/Main.cpp:109-116)


def fk64(angles: np.ndarray) -> np.ndarray:
    """Independent float64 FK of the reference scene: node k = parent * Rx Ry Rz * T(1,0,0)."""
    def rot(a, b, c):
        ca, sa, cb, sb, cc, sc = np.cos(a), np.sin(a), np.cos(b), np.sin(b), np.cos(c), np.sin(c)
        rx = np.array([[1, 0, 0], [0, ca, -sa], [0, sa, ca]])
        ry = np.array([[cb, 0, sb], [0, 1, 0], [-sb, 0, cb]])
        rz = np.array([[cc, -sc, 0], [sc, cc, 0], [0, 0, 1]])
        return rx @ ry @ rz
    R = [np.eye(3)]
    p = [np.zeros(3)]
    out = []
    for k in range(1, 8):
        Rl = rot(*angles[3 * (k - 1):3 * k])
        Rw = R[PARENTS[k]] @ Rl
        pw = p[PARENTS[k]] + Rw[:, 0] * 1.0
        R.append(Rw)
        p.append(pw)
        out.append(pw)
    return np.concatenate(out)


def make_fk_kat(sheets: dict) -> None:
    degs, poss, ids, dropped = [], [], [], []
    for n in (1, 2, 3):
        d = numeric_rows(sheets[f"DEGREES_{n}"], 21)
        p = numeric_rows(sheets[f"POSITIONS_{n}"], 21)
        for r in sorted(set(d) & set(p)):
            err = np.max(np.abs(fk64(d[r]) - p[r]))
            if err < 1e-4:
                degs.append(d[r])
                poss.append(p[r])
                ids.append((n, r))
            else:
                dropped.append((n, r))
    np.savez_compressed(
        HERE / "fk_kat.npz",
        degrees=np.array(degs, dtype=np.float32),
        positions=np.array(poss, dtype=np.float32),
        ids=np.array(ids, dtype=np.int32),
        dropped=np.array(dropped, dtype=np.int32),
    )
    print(f"fk_kat: kept {len(ids)} rows, dropped {len(dropped)} stale rows: {dropped}")


RESET_TARGETS = np.array([[0.75, 1.0, -2.5], [-0.75, 1.0, -2.5], [0.0, 0.0, -2.5]])


def make_distance_kat(sheets: dict) -> None:
    p = numeric_rows(sheets["POSITIONS_1"], 21)
    d = numeric_rows(sheets["DISTANCE_1"], 1)
    a = numeric_rows(sheets["DEGREES_1"], 21)
    rows = sorted(set(p) & set(d) & set(a))
    stale = [r for r in rows if np.max(np.abs(fk64(a[r]) - p[r])) >= 1e-4]  # see make_fk_kat
    rows = [r for r in rows if r not in stale]
    eff = np.array([p[r][12:21].reshape(3, 3) for r in rows])  # nodes 5, 6, 7 (effectors)
    dist = np.array([d[r][0] for r in rows])
    recomputed = np.linalg.norm(eff - RESET_TARGETS[None], axis=2).sum(axis=1)
    print(f"distance_kat: {len(rows)} rows (dropped stale {stale}), max |logged - recomputed| = {np.max(np.abs(recomputed - dist)):.3g}")
    np.savez_compressed(HERE / "distance_kat.npz", effector_positions=eff.astype(np.float32),
                        degrees=np.array([a[r] for r in rows], dtype=np.float32),
                        distance=dist.astype(np.float32), rows=np.array(rows, dtype=np.int32),
                        targets=RESET_TARGETS.astype(np.float32))


def make_frames(sheets: dict) -> None:
    rows = sheets["FRAMES_3"]
    vals = [int(float(rows[r]["A"])) for r in range(2, 22)]
    summary = {k: float(rows[r]["A"]) for k, r in (("mean", 23), ("max", 24), ("min", 25))}
    with open(HERE / "frames3.json", "w") as f:
        json.dump({"source": "results.xlsx FRAMES_3!A2:A21 (iteration 3 = HEAD code), summary A23:A25",
                   "frames": vals, "summary": summary,
                   "setup": "21-DOF scene, N=16384 particles, 15 PSO iterations per frame, "
                            "converged when sum of effector distances <= 0.025"}, f, indent=1)
    print("frames3:", vals, summary)


PROBE = r'''
#include <rocrand/rocrand_xorwow.h>
#include <cstdio>
#include <cstdlib>
struct probe : rocrand_device::xorwow_engine {
    probe(unsigned d, const unsigned* v) : xorwow_engine(0, 0, 0) {
        m_state.d = d;
        for (int i = 0; i < 5; ++i) m_state.x[i] = v[i];
    }
};
int main(int argc, char** argv) {
    // argv: n, then d v0..v4 per state
    int n = atoi(argv[1]);
    for (int a = 2; a + 5 < argc; a += 6) {
        unsigned d = strtoul(argv[a], 0, 10), v[5];
        for (int i = 0; i < 5; ++i) v[i] = strtoul(argv[a + 1 + i], 0, 10);
        probe e(d, v);
        for (int i = 0; i < n; ++i) printf("%u%c", e.next(), i + 1 == n ? '\n' : ' ');
    }
    return 0;
}
'''


def curand_init_state(seed: int):
    """cuRAND curand_init(seed, 0, 0) XORWOW state (see oracle/ikpso_oracle.c)."""
    m = 0xFFFFFFFF
    s0 = (seed & m) ^ 0xAAD26B49
    s1 = ((seed >> 32) & m) ^ 0xF7DCEFDD
    t0 = (1099087573 * s0) & m
    t1 = (2591861531 * s1) & m
    d = (6615241 + t1 + t0) & m
    v = [(123456789 + t0) & m, 362436069 ^ t0, (521288629 + t1) & m, 88675123 ^ t1, (5783321 + t0) & m]
    return d, v


def make_xorwow() -> None:
    seeds = [0, 1, 2, 3, 255, 1023, (1 << 32) + 5]
    n = 64
    with tempfile.TemporaryDirectory() as td:
        src = Path(td) / "probe.cpp"
        exe = Path(td) / "probe"
        src.write_text(PROBE)
        subprocess.run(["/opt/rocm/bin/hipcc", "-O1", "-x", "c++", str(src), "-o", str(exe),
                        "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"], check=True)
        args = [str(n)]
        states = []
        for s in seeds:
            d, v = curand_init_state(s)
            states.append([d] + v)
            args += [str(d)] + [str(x) for x in v]
        out = subprocess.run([str(exe)] + args, check=True, capture_output=True, text=True).stdout
    draws = [[int(x) for x in line.split()] for line in out.strip().splitlines()]
    with open(HERE / "xorwow_rocrand.json", "w") as f:
        json.dump({"source": "rocrand_device::xorwow_engine::next() (rocrand_xorwow.h), from the cuRAND "
                             "curand_init(seed,0,0) states of these seeds",
                   "seeds": seeds, "states": states, "draws": draws}, f)
    print(f"xorwow_rocrand: {len(seeds)} states x {n} draws")


def main() -> int:
    if not XLSX.exists():
        print(f"{XLSX} not found (the reference is only mounted in the build container)", file=sys.stderr)
        return 1
    sheets = read_sheets(XLSX)
    make_fk_kat(sheets)
    make_distance_kat(sheets)
    make_frames(sheets)
    make_xorwow()
    return 0


if __name__ == "__main__":
    sys.exit(main())
