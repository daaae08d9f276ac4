#!/usr/bin/env python3
"""Per-kernel VGPR / scratch / spill / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage.  usage: resource_usage.py FILE.hip [extra hipcc flags]"""
import re
import subprocess
import sys
from pathlib import Path

CSRC = Path(__file__).resolve().parents[1] / "inverse-kinematics-pso-research_amd" / "csrc"
src = sys.argv[1]
flags = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize", f"-I{CSRC}",
       f"-I{CSRC.parents[1] / 'include'}", "-c", str(CSRC / src), "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage"] + flags
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|SGPRs Spill|"
                  r"Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split()[0] + ("_spill" if "Spill" in k else "")] = v
for r in rows:
    n = re.sub(r"^_ZN5ikpso\d+", "", r["name"])
    n = re.sub(r"EEEvNS_11ChainConsts.*|EEvNS_11ChainConsts.*|EvNS.*", "", n)
    print(f"{n:60s} vgpr={r.get('VGPRs','?'):>4} scratch={r.get('ScratchSize','?'):>5} "
          f"vspill={r.get('VGPRs_spill','0'):>4} sspill={r.get('SGPRs_spill','0'):>4} occ={r.get('Occupancy','?')}")
