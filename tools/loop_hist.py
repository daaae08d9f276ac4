"""Opcode histogram of the largest loop in one kernel of a hipcc -S listing.

usage: python tools/loop_hist.py FILE.s KERNEL_SUBSTRING
Finds the kernel's body, the back-edge with the longest span (label ... branch
to that label) and prints instruction counts by opcode and by class.
"""
import collections
import re
import sys

path, key = sys.argv[1], sys.argv[2]
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.size") or lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = i
best = None
for i, l in enumerate(body):
    m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        span = i - labels[m.group(1)]
        if best is None or span > best[1] - best[0]:
            best = (labels[m.group(1)], i)
lo, hi = best
ops = collections.Counter()
for l in body[lo:hi + 1]:
    s = l.strip()
    if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
        continue
    ops[s.split()[0]] += 1
total = sum(ops.values())
cls = collections.Counter()
for op, n in ops.items():
    c = "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else "mem"
    cls[c] += n
print(f"loop lines {lo}-{hi}: {total} instructions", dict(cls))
for op, n in ops.most_common(60):
    print(f"{n:6d} {op}")
