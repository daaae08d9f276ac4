#!/usr/bin/env python3
"""Which FAST ingredient widens tier B?  (VERDICT r4 "next" 1)

FAST arithmetic differs from the oracle (the reference's operation order,
src/kernel.cu:153-189,279-327) by several ingredients; each attribution build
removes one (ikpso_device.h: IKPSO_FAST_REV, IKPSO_FAST_HW_TRIG,
IKPSO_FAST_TIP_BACKWARD; tools/build_variants.sh).  This script

  run LIB...   (GPU box) solves the tier-B batches of tests/golden/tierb_config{3,5}.npz
               -- 256 swarms of config 3, 128 of config 5, 500 iterations -- with every
               library and writes gpurun_out/tierb_attr_config{3,5}.npz;
  analyze [TIMINGS.json]  (here) compares each library's answers with the oracle's,
               next to the oracle's own FMA on/off envelope on the same swarms, runs the
               stated tests (tests/tierb.py: stat_tests) and writes
               profiles/r05/tier_b_attribution.json.

Test infrastructure (reads the oracle's fixtures)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "tools"), str(ROOT / "tests"), str(ROOT / "oracle"),
                str(ROOT / "inverse-kinematics-pso-research_amd")]
import numpy as np

import ikpso

BATCH = {3: 256, 5: 128}


def run(libs):
    import torch
    from variant_bench import make_solver, open_lib

    for cfg, B in BATCH.items():
        wl = ikpso.workload(cfg)
        P, I, D = wl.particles, wl.iterations, wl.dof
        tg = torch.from_numpy(np.ascontiguousarray(wl.targets(0, B))).cuda()
        out = {}
        for p in libs:
            lib = open_lib(p)
            h, keep = make_solver(lib, wl, P, I)
            o = [torch.empty((B, D), device="cuda"), torch.empty(B, device="cuda"), torch.empty(B, device="cuda")]
            assert lib.ikpso_solver_seed(h, B, 0, 0, None) == 0
            assert lib.ikpso_solve_batch(h, tg.data_ptr(), None, B, I, o[0].data_ptr(), o[1].data_ptr(),
                                         o[2].data_ptr(), None) == 0
            assert lib.ikpso_solver_sync(h) == 0
            torch.cuda.synchronize()
            name = Path(p).stem
            out[f"{name}__angles"], out[f"{name}__fitness"], out[f"{name}__residual"] = (t.cpu().numpy() for t in o)
            lib.ikpso_solver_destroy(h)
            print(f"config {cfg} {name}: mean fitness {out[f'{name}__fitness'].mean():.6f}", flush=True)
        (ROOT / "gpurun_out").mkdir(exist_ok=True)
        np.savez(ROOT / "gpurun_out" / f"tierb_attr_config{cfg}.npz", **out)


def analyze(timings=None):
    from tierb import envelope, load_fixture, stat_tests, tier_b_distances, tier_b_report

    res = {"note": __doc__.strip().splitlines()[0], "timings": timings}
    for cfg in BATCH:
        wl = ikpso.workload(cfg)
        fx = load_fixture(cfg)
        env = envelope(wl.chain, fx)
        block = {"envelope": tier_b_report(*env)}
        z = np.load(ROOT / "gpurun_out" / f"tierb_attr_config{cfg}.npz")
        for name in sorted({k.split("__")[0] for k in z.files}):
            ang, fit, r = z[f"{name}__angles"], z[f"{name}__fitness"], z[f"{name}__residual"]
            d = tier_b_distances(wl.chain, ang, fit, r, fx["ref_angles"], fx["ref_fitness"], fx["ref_residual"])
            block[name] = {"distribution": tier_b_report(*d),
                           "tests": stat_tests(d, env, fit, fx["ref_fitness"])}
        res[f"config{cfg}"] = block
    dst = ROOT / "profiles" / "r05" / "tier_b_attribution.json"
    dst.parent.mkdir(parents=True, exist_ok=True)
    dst.write_text(json.dumps(res, indent=1) + "\n")
    for cfg in BATCH:
        b = res[f"config{cfg}"]
        for name, v in b.items():
            dist = v if name == "envelope" else v["distribution"]
            print(f"config {cfg} {name:24s} p90 df/f {dist['rel_fitness']['p90']:.2e}  res {dist['residual_abs']['p90']:.2e}"
                  f"  pos {dist['effector_pos_abs']['p90']:.2e}  within {dist['frac_rel_le_1e-3']:.3f} "
                  f"{dist['frac_res_le_1e-3']:.3f} {dist['frac_pos_le_1e-2']:.3f}"
                  + ("" if name == "envelope" else f"  pass {v['tests']['pass']}"))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2:])
    else:
        analyze(json.loads(Path(sys.argv[2]).read_text()) if len(sys.argv) > 2 else None)
