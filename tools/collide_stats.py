#!/usr/bin/env python3
"""What the collider term of the fitness does on the GPU (SURVEY §8(f2);
src/kernel.cu:104-136): run with an IKPSO_COLLIDE_STATS build of the library
(tools/build_variants.sh REF7_ONLY collide_stats -DIKPSO_COLLIDE_STATS=1), which
counts, per solve, the box/collider pairs through the inline sphere test and
how many pass it, the pairs through the quaternion sphere test, the GJK calls,
their loop trips summed over lanes and over waves (the SIMD's view), and hits.

  IKPSO_LIB=vlib6/collide_stats.so IKPSO_ALLOW_STALE=1 \\
      python tools/collide_stats.py [SWARMS] [ITERS] [SCENE] [OUT.json]

SCENE: init03 (initColliders boxes 0 and 3, src/Main.cpp:537-559, which leave the
reset pose clear: bench.py's collide leg), init4 (all four), far4 (all four moved
1000 units away)."""
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "inverse-kinematics-pso-research_amd"))
import numpy as np
import torch

import ikpso
from ikpso import _abi

NAMES = ["pre", "pre_pass", "exact", "exact_pass", "gjk_lane_trips", "gjk_wave_trips", "gjk_hits", "wave_calls"]


def scene(name):
    boxes = ikpso.init_colliders(4)
    if name == "init03":
        return boxes[[0, 3]]
    if name == "far4":
        boxes["pos"] += 1000.0
    return boxes


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    I = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    name = sys.argv[3] if len(sys.argv) > 3 else "init03"
    lib = _abi.load()
    fn = lib.ikpso_debug_collide_stats
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    wl = ikpso.workload(3)
    P, J = wl.particles, wl.chain.shape[0] - 1
    boxes = scene(name)
    tg = torch.from_numpy(np.ascontiguousarray(wl.targets(0, B))).cuda()
    s = ikpso.BatchSolver(wl.chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), colliders=boxes)
    s.seed(B)
    buf = np.zeros(8, dtype=np.uint64)
    assert fn(buf.ctypes.data, 1) == 0  # clear
    ang, fit, res = (t.cpu().numpy() for t in s.solve(tg, iterations=I))
    assert fn(buf.ctypes.data, 1) == 0
    c = dict(zip(NAMES, (int(v) for v in buf)))
    evals = B * P * (I + 1)  # the initial evaluation and one per iteration
    wave_nodes = evals // 64 * J
    out = {
        "workload": f"config 3 scene, {B} swarms x {P} particles x {I} iterations, colliders {name} "
                    f"({len(boxes)} boxes), FAST arithmetic, kernel {s.kernel}",
        "counters": c,
        "evaluations": evals,
        "pre_pass_rate": c["pre_pass"] / max(c["pre"], 1),
        "exact_pass_rate_of_called": c["exact_pass"] / max(c["exact"], 1),
        "gjk_calls_per_evaluation": c["exact_pass"] / evals,
        "gjk_trips_per_call": c["gjk_lane_trips"] / max(c["exact_pass"], 1),
        "gjk_simt_efficiency": c["gjk_lane_trips"] / max(64 * c["gjk_wave_trips"], 1),
        "gjk_hit_rate": c["gjk_hits"] / max(c["exact_pass"], 1),
        "wave_node_call_share": c["wave_calls"] / max(wave_nodes, 1),
        "calls_per_wave_evaluation": c["wave_calls"] / max(evals // 64, 1),
        "answers_colliding": int((fit > 1e30).sum()),
        "mean_fitness": float(fit[fit < 1e30].mean()) if (fit < 1e30).any() else None,
        "note": "pre: node/collider pairs through the inline sphere test in the FK pass (every node of every "
                "evaluation); exact: pairs through the quaternion test in node_collides, which the fitness's "
                "finish calls for the near nodes after the pass -- in the swarm step only for lanes whose collision-free "
                "value could still improve their local best -- until the first hit; calls_per_wave_evaluation: "
                "node_collides calls a wave makes per evaluation (one per trip of finish's loop over the lanes' "
                "near nodes; wave_node_call_share = the same per node); gjk_simt_efficiency: GJK loop trips summed "
                "over lanes / (64 x trips summed over waves)",
    }
    s.close()
    text = json.dumps(out, indent=1)
    print(text)
    if len(sys.argv) > 4:
        Path(sys.argv[4]).write_text(text + "\n")


if __name__ == "__main__":
    main()
