#!/usr/bin/env python3
"""Tier-B fixtures: the CPU oracle's answers for the FAST parity batches of
BASELINE configs 3 and 5 (SURVEY.md §8(c) tier B), each solved twice --

  ref  the oracle as the parity checker builds it (-ffp-contract=off): the
       reference's algorithm, src/kernel.cu:153-327, in its operation order;
  fma  the same source with FMA contraction (-mfma -ffp-contract=fast): a second
       valid fp32 evaluation of the same solves, one rounding apart -- the
       envelope two valid evaluations span after 500 chaotic iterations.

  tierb_config3.npz  256 swarms x 1024 particles x 500 iterations (config 3's
                     targets and global seeds, swarms 0..255)
  tierb_config5.npz  128 swarms x 4096 particles x 500 iterations (config 5's
                     20-joint chain with its soft-limit penalty, swarms 0..127)
  tierb_collide.npz  256 swarms of config 3 (1024 particles x 500 iterations) with
                     the reference's initColliders boxes 0 and 3 (src/Main.cpp:537-559,
                     the fitness term src/kernel.cu:104-136): the bench's collide leg

Each holds angles [B, D], fitness [B], residual [B] for both builds.  The GPU
parity tests (tests/test_gpu_parity.py, tests/test_gpu_config5.py) compare the
GPU's FAST answers with `ref` and the `fma` answers with `ref` on the same
swarms; tests/test_tierb_fixtures.py re-solves a few swarms with the oracle and
checks they reproduce bit for bit.  Test infrastructure (imports oracle/);
about 30 minutes on 8 threads (collide: ~15).  usage: make_tierb.py [3] [5] [collide]
"""
from __future__ import annotations

import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "inverse-kinematics-pso-research_amd")]

import ikpso  # noqa: E402
import oracle  # noqa: E402

BATCH = {3: 256, 5: 128, "collide": 256}


def solve(cfg, B: int, lib, first: int = 0):
    wl = ikpso.workload(3 if cfg == "collide" else cfg)
    kw = dict(limit_weight=wl.limit_weight, soft_lo=wl.soft_lo, soft_hi=wl.soft_hi)
    if cfg == "collide":
        kw["colliders"] = ikpso.init_colliders(4)[[0, 3]]
    rng = oracle.init_generators(B * wl.particles, first * wl.particles)
    return oracle.solve_batch(wl.chain, wl.targets(first, B), None, wl.particles, wl.iterations, rng, threads=0,
                              lib=lib, **kw)


def main():
    cfgs = [a if a == "collide" else int(a) for a in sys.argv[1:]] or [3, 5, "collide"]
    for cfg in cfgs:
        B = BATCH[cfg]
        out = {"swarms": np.int64(B)}
        for name, lib in (("ref", oracle.load()), ("fma", oracle.load_fma())):
            t0 = time.time()
            a, f, r = solve(cfg, B, lib)
            out.update({f"{name}_angles": a, f"{name}_fitness": f, f"{name}_residual": r})
            print(f"config {cfg} {name}: {B} swarms in {time.time() - t0:.0f} s", flush=True)
        np.savez_compressed(HERE / (f"tierb_{cfg}.npz" if cfg == "collide" else f"tierb_config{cfg}.npz"), **out)


if __name__ == "__main__":
    main()
