#!/usr/bin/env python3
"""Collect gpurun_out/prof_* (tools/gpu_profile.sh) into profiles/<round>/ and
refresh profiles/valu_per_update.json (used by bench.py's roofline).
usage: update_profiles.py ROUND_DIR SWARMS [KERNEL_SUBSTRING]"""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
out_dir = ROOT / "profiles" / sys.argv[1]
swarms = int(sys.argv[2])
pat = sys.argv[3] if len(sys.argv) > 3 else "k_swarm_resident"
out_dir.mkdir(parents=True, exist_ok=True)
src = ROOT / "gpurun_out"
shutil.copy(src / "prof_trace" / "run_kernel_stats.csv", out_dir / "kernel_stats.csv")
counters = {}
for name in ("valu", "fetch", "write", "cycles"):
    rows = list(csv.DictReader(open(src / f"prof_{name}" / "run_counter_collection.csv")))
    agg = collections.OrderedDict()
    for r in rows:
        key = (r["Dispatch_Id"], r["Kernel_Name"], r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"],
               r["VGPR_Count"], r["SGPR_Count"], r["Scratch_Size"])
        agg.setdefault(key, collections.OrderedDict())
        agg[key][r["Counter_Name"]] = agg[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    cn = sorted({c for v in agg.values() for c in v})
    with open(out_dir / f"pmc_{name}.csv", "w") as f:
        w = csv.writer(f)
        w.writerow(["dispatch", "kernel", "grid", "wg", "lds", "vgpr", "sgpr", "scratch"] + cn)
        for k, v in agg.items():
            w.writerow(list(k) + [v.get(c, "") for c in cn])
    big = [v for k, v in agg.items() if pat in k[1] and int(k[2]) == swarms * 1024]
    counters[name] = big[-1]
updates = swarms * 1024 * 500
valu = counters["valu"]["SQ_INSTS_VALU"] * 64 / updates
fb = counters["fetch"]["FETCH_SIZE"] * 1024 * 2  # KiB; x2: gfx950 FETCH_SIZE counts half a streaming read
wb = counters["write"]["WRITE_SIZE"] * 1024
cyc = counters["cycles"]
res = {
    "valu_lane_instr_per_update": round(valu, 1),
    "hbm_bytes_per_update": round((fb + wb) / updates, 4),
    "wave_cycle_split": {k: round(cyc[k] / cyc["SQ_WAVE_CYCLES"], 3)
                         for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")},
    "effective_clock_ghz": None,
    "source": f"rocprofv3 --pmc SQ_INSTS_VALU / FETCH_SIZE / WRITE_SIZE / cycles (separate passes), {pat}, "
              f"{swarms} swarms x 1024 particles x 500 iterations; profiles/{sys.argv[1]}/pmc_*.csv. "
              "lane-instr/update = SQ_INSTS_VALU * 64 / updates; bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB*1024 / updates",
    "fetch_bytes": fb, "write_bytes": wb, "updates": updates,
}
stats = list(csv.DictReader(open(out_dir / "kernel_stats.csv")))
k = [r for r in stats if pat in r["Name"]]
if k:
    ns = float(k[0]["MaxNs"])
    res["effective_clock_ghz"] = round(counters["valu"]["GRBM_GUI_ACTIVE"] / 8 / ns, 3)
json.dump(res, open(ROOT / "profiles" / "valu_per_update.json", "w"), indent=1)
print(json.dumps(res, indent=1))
