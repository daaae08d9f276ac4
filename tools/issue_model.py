#!/usr/bin/env python3
"""Issue-cycle model of a kernel's hot loop: the loop's VALU opcode histogram
(hipcc -S listing) weighted by the gfx950 per-opcode issue costs measured by
tools/probes/valu_probe.hip (profiles/r02/valu_issue_costs.txt).

usage: issue_model.py FILE.s KERNEL_SUBSTRING
Prints VALU instructions per iteration and the modelled SIMD cycles per
wave-iteration (the sum of issue costs), by cost class.
"""
import collections
import re
import sys

# cycles per wave64 op per SIMD (valu_probe.hip, 4 waves per SIMD)
COST4 = ("v_lshlrev_b32", "v_add3_u32", "v_cvt_f32_u32", "v_cvt_f32_i32", "v_cvt_u32_f32", "v_cvt_i32_f32",
         "v_med3_f32", "v_max_f32", "v_min_f32", "v_max3_f32", "v_min3_f32", "v_bfe_i32", "v_bfe_u32",
         "v_alignbit_b32", "v_lshl_add_u32", "v_lshl_or_b32", "v_xad_u32", "v_lshlrev_b64", "v_lshl_add_u64",
         "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_readlane_b32", "v_writelane_b32", "v_perm_b32",
         "v_and_or_b32", "v_or3_b32", "v_cndmask_b32")
TRANS = ("v_sin_f32", "v_cos_f32", "v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32")
# fp64 and packed-fp32 forms (round 4, profiles/r04/valu_issue_costs.txt): the REFERENCE sincos runs in fp64
COSTF64 = {"v_fma_f64": 4.79, "v_fmac_f64": 4.79, "v_mul_f64": 4.41, "v_add_f64": 4.09, "v_cvt_f64_f32": 4.11,
           "v_cvt_f32_f64": 4.12, "v_pk_mul_f32": 4.09, "v_pk_fma_f32": 4.11, "v_pk_add_f32": 4.1,
           "v_rndne_f32": 4.06, "v_mov_b64": 4.1}


# ordinary ops measured individually by the probe (VGPR operands); others 2.2
COST2 = {"v_mul_f32": 2.17, "v_fmac_f32": 2.29, "v_fma_f32": 2.23, "v_fmaak_f32": 2.05, "v_fmamk_f32": 2.12,
         "v_sub_f32": 2.19, "v_xor_b32": 2.45, "v_bitop3_b32": 2.48, "v_lshrrev_b32": 2.16, "v_add_u32": 2.30,
         "v_and_b32": 2.08, "v_mov_b32": 2.12}


def cost(op):
    base = re.sub(r"_e(32|64)$|_dpp$|_sdwa$", "", op)
    if base in TRANS:
        return 8.1, "trans"
    if base in COSTF64:
        return COSTF64[base], "4-cycle"
    if base in COST4:
        return 4.1, "4-cycle"
    return COST2.get(base, 2.2), "2-cycle"


def hot_loop(path, key):
    lines = open(path).read().splitlines()
    s = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l)
    e = next(i for i in range(s + 1, len(lines)) if lines[i].startswith("\t.size") or lines[i].startswith(".Lfunc_end"))
    body = lines[s:e]
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\w+):", l))}
    # the innermost loop with the most VALU instructions: a back-edge whose span holds no other back-edge target
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    def valu(lo, hi):
        return sum(1 for l in body[lo:hi + 1] if l.strip().startswith("v_"))
    lo, hi = max(loops, key=lambda t: (valu(*t) if valu(*t) < 0.6 * valu(0, len(body) - 1) else -1))
    return body[lo:hi + 1]


def model(path, key):
    """The hot loop's VALU mix and modelled issue cycles (a dict for profiles/valu_per_update.json)."""
    loop = hot_loop(path, key)
    ops = collections.Counter(l.split()[0] for l in loop if l.strip().startswith("v_"))
    n = collections.Counter()
    cyc = collections.Counter()
    for op, k in ops.items():
        c, cls = cost(op)
        cyc[cls] += c * k
        n[cls] += k
    total_n, total_c = sum(n.values()), sum(cyc.values())
    return {"loop_valu_instr": total_n, "loop_issue_cycles": round(total_c, 1),
            "mean_cycles_per_instr": round(total_c / total_n, 4),
            "by_class": {k: {"instr": n[k], "cycles": round(cyc[k], 1)} for k in ("2-cycle", "4-cycle", "trans")},
            "costs": "tools/probes/valu_probe.hip (profiles/r02/valu_issue_costs.txt): 2.05-2.48 (measured per op) / "
                     "4.1 / 8.1 SIMD cycles per wave64 op; hot loop = the kernel's PSO iteration loop in its hipcc -S listing"}


def main():
    loop = hot_loop(sys.argv[1], sys.argv[2])
    ops = collections.Counter(l.split()[0] for l in loop if l.strip().startswith("v_"))
    cyc = collections.Counter()
    n = collections.Counter()
    for op, k in ops.items():
        c, cls = cost(op)
        cyc[cls] += c * k
        n[cls] += k
    total = sum(cyc.values())
    print(f"VALU instructions per wave-iteration: {sum(n.values())}  modelled issue cycles: {total:.0f}")
    for cls in ("2-cycle", "4-cycle", "trans"):
        print(f"  {cls:8s} {n[cls]:6d} instr  {cyc[cls]:8.0f} cycles")
    other = collections.Counter(l.split()[0] for l in loop if l.strip() and l.strip()[0] in "sdgf"
                                and not l.strip().startswith(";"))
    print("  memory/scalar:", {k: v for k, v in other.items() if k.startswith(("ds_", "global_", "scratch_", "flat_",
                                                                                 "s_waitcnt", "s_barrier"))})


if __name__ == "__main__":
    main()
