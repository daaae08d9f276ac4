#!/usr/bin/env python3
"""Collect gpurun_out/<name>_* (tools/gpu_profile.sh) into profiles/<round>/ and
record the kernel's per-update counters in profiles/valu_per_update.json
(keyed by the solver's kernel name; bench.py's roofline reads it).
usage: update_profiles.py ROUND NAME KERNEL_SUBSTRING KEY UPDATES_PER_DISPATCH [TU ISA_SYMBOL_SUBSTRING]
With TU (an ikpso_inst_*.hip unit) the unit is compiled to its ISA listing with the
library's flags and tools/issue_model.py's issue-cycle model of the kernel's hot
loop is stored with the counters (bench.py's issue-slot roofline reads it)."""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
rnd, name, pat, key, upd = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5])
tu, sym = (sys.argv[6], sys.argv[7]) if len(sys.argv) > 7 else (None, None)
out_dir = ROOT / "profiles" / rnd
out_dir.mkdir(parents=True, exist_ok=True)
src = ROOT / "gpurun_out"
shutil.copy(src / f"{name}_trace" / "run_kernel_stats.csv", out_dir / f"{name}_kernel_stats.csv")
counters = {}
for pas in ("valu", "fetch", "write", "cycles", "waits"):
    if not (src / f"{name}_{pas}" / "run_counter_collection.csv").exists():  # (waits: round 6 on)
        continue
    rows = list(csv.DictReader(open(src / f"{name}_{pas}" / "run_counter_collection.csv")))
    agg = collections.OrderedDict()
    for r in rows:
        k = (r["Dispatch_Id"], r["Kernel_Name"], r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"],
             r["VGPR_Count"], r["SGPR_Count"], r["Scratch_Size"])
        agg.setdefault(k, collections.OrderedDict())
        agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    cn = sorted({c for v in agg.values() for c in v})
    with open(out_dir / f"{name}_pmc_{pas}.csv", "w") as f:
        w = csv.writer(f)
        w.writerow(["dispatch", "kernel", "grid", "wg", "lds", "vgpr", "sgpr", "scratch"] + cn)
        for k, v in agg.items():
            w.writerow(list(k) + [v.get(c, "") for c in cn])
    # the largest dispatch of the kernel (the batch, not the single-solve timing runs)
    big = max((k for k in agg if pat in k[1]), key=lambda k: int(k[2]))
    counters[pas] = agg[big]
valu = counters["valu"]["SQ_INSTS_VALU"] * 64 / upd
trans = counters["valu"].get("SQ_INSTS_VALU_TRANS_F32")  # v_sin/v_cos/...: 4 issue slots each on gfx950
trans = None if trans is None else trans * 64 / upd
fb = counters["fetch"]["FETCH_SIZE"] * 1024 * 2  # KiB; x2: gfx950 FETCH_SIZE counts half a streaming read
wb = counters["write"]["WRITE_SIZE"] * 1024
cyc = counters["cycles"]
res = {
    "valu_lane_instr_per_update": round(valu, 1),
    "trans_lane_instr_per_update": None if trans is None else round(trans, 1),
    "hbm_bytes_per_update": round((fb + wb) / upd, 4),
    "wave_cycle_split": {k: round(cyc[k] / cyc["SQ_WAVE_CYCLES"], 3)
                         for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")},
    "source": f"rocprofv3 --pmc SQ_INSTS_VALU (+ SQ_INSTS_VALU_TRANS_F32) / FETCH_SIZE / WRITE_SIZE / cycles (separate passes) of {pat}, "
              f"{upd} particle-updates per dispatch; profiles/{rnd}/{name}_pmc_*.csv. lane-instr/update = "
              "SQ_INSTS_VALU * 64 / updates; bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB*1024 / updates",
    "fetch_bytes": fb, "write_bytes": wb, "updates": upd,
    # ikpso_build_id() of the library the counters were collected on (tools/gpu_profile.sh)
    "build_id": (src / f"{name}_build_id.txt").read_text().strip() if (src / f"{name}_build_id.txt").exists()
    else None,
}
if tu:
    import subprocess
    sys.path.insert(0, str(ROOT / "tools"))
    import issue_model
    csrc = ROOT / "inverse-kinematics-pso-research_amd" / "csrc"
    asm = Path("/tmp") / (Path(tu).stem + ".s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
                    f"-I{csrc}", f"-I{ROOT / 'include'}", "--cuda-device-only", "-S", str(csrc / tu), "-o", str(asm)],
                   check=True, capture_output=True)
    res["issue_model"] = dict(issue_model.model(str(asm), sym), tu=tu, symbol=sym)
db_path = ROOT / "profiles" / "valu_per_update.json"
db = json.loads(db_path.read_text()) if db_path.exists() else {}
if "valu_lane_instr_per_update" in db:  # old single-kernel format
    db = {"swarm_resident<ref_tree7>": db}
db[key] = res
db_path.write_text(json.dumps(db, indent=1) + "\n")
print(json.dumps(res, indent=1))
