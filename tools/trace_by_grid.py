#!/usr/bin/env python3
"""Per-(kernel, grid) dispatch statistics of a rocprofv3 --kernel-trace run.

rocprofv3's --stats summary averages every dispatch of a kernel symbol; bench.py's
default run launches config 3's k_swarm_resident<TopoRef7, 0, 200> with 4096
swarms (the headline steps) and with 8192 (config 4's leg), so the headline
kernel's average is read here per grid size (the number that must agree with the
line's HIP-event kernel_ms).  usage: trace_by_grid.py RUN_KERNEL_TRACE.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print(f"{'kernel':70s} {'grid':>9s} {'wg':>5s} {'calls':>5s} {'avg ms':>10s} {'min ms':>10s} {'max ms':>10s}")
for (name, grid, wg), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{name[:70]:70s} {grid:9d} {wg:5d} {len(v):5d} {sum(v) / len(v):10.3f} {min(v):10.3f} {max(v):10.3f}")
