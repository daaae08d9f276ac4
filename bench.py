#!/usr/bin/env python3
"""Throughput of the PSO inverse-kinematics hot path on MI355X.

One step = one batch of independent IK solves (one swarm per target) on every
rank: BASELINE config 3 per GPU -- the reference's 7-joint (21-DOF) scene,
4096 perturbed targets, 1024 particles per swarm, 500 PSO iterations -- then
one all-gather of the per-swarm results (RCCL over xGMI) and a copy of the
gathered results to the host.  Inputs (targets) are resident in HBM before the
timed region.  Weak scaling: per-GPU work is fixed, N GPUs solve N x 4096
targets (N = 8 is 32768 targets; `--swarms-per-gpu 8192` gives config 4's
65536).  Generator seeds are global (swarm b, particle i: curand_init(b*1024+i)).

With the default config 3 the same run also times, every rank, the other
BASELINE lines under "legs": config 4's shard (8192 targets per GPU, so N = 8
is the named 65536), config 5 at its named size (8192 targets of the 20-joint
chain over all GPUs) and the DH arm (dh7); `--extra-steps 0` skips them.

Prints ONE JSON line on rank 0 (see DESIGN.md for every field).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "inverse-kinematics-pso-research_amd"))

# MI355X constants (MI355X_MICROARCH.md "Chip-level parameters")
HBM_PEAK_GBS = 8000.0
CUS, SIMDS, LANES_PER_CLK, CLOCK_GHZ = 256, 4, 32, 2.4
VALU_PEAK_TINSTR = CUS * SIMDS * LANES_PER_CLK * CLOCK_GHZ / 1e3  # VALU lane-instructions/s, 78.6 T
# algorithmic bytes per particle-update = 20*D + 8 (x, v, pbest read; x, v written; pbest
# fitness r/w): 428 B at D = 21, 1208 B at D = 60


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="3", choices=["2", "3", "4", "5", "dh7", "dh7-nofold", "dh7-locked"],
                    help="BASELINE config: 2 = one swarm (latency), 3 = 4096 targets per GPU (default), "
                         "4 = 65536 targets over all GPUs, 5 = 20-joint chain, 8192 targets over all GPUs, "
                         "4096 particles, penalty; dh7* = the 7-joint iiwa DH arm, 4096 targets per GPU, with "
                         "its joint-axis mask (dh7: folded chain; dh7-nofold: Euler kernels) or locked axes")
    ap.add_argument("--swarms-per-gpu", type=int, default=None)
    ap.add_argument("--particles", type=int, default=None)
    ap.add_argument("--iterations", type=int, default=None)
    ap.add_argument("--arith", choices=["fast", "reference"], default="fast")
    ap.add_argument("--colliders", choices=["none", "init03", "init4", "far4"], default="none",
                    help="config 3 with the reference's initColliders boxes (src/Main.cpp:537-559): 0 and 3, all "
                         "four, or all four moved 1000 units away (the collider kernel with nothing near)")
    ap.add_argument("--kernel", choices=["auto", "resident", "coop", "streaming"], default="auto",
                    help="kernel family (auto: resident if the swarm fits one workgroup, else cooperative)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = every CPU in this process's affinity mask)")
    ap.add_argument("--reference-steps", type=int, default=3,
                    help="after the FAST legs, time this many steps of the same workload in REFERENCE arithmetic "
                         "(the bit-exact path; rank 0, configs 3/4; 0 = skip)")
    ap.add_argument("--extra-legs", default="4,5,dh7,collide",
                    help="with the default config 3: also time these BASELINE lines in the same run and print them "
                         "under 'legs' (4 = config 4's 8192 targets per GPU, 5 = config 5, dh7 = the DH arm, "
                         "collide = config 3 with the reference's collider boxes)")
    ap.add_argument("--extra-steps", type=int, default=2, help="timed steps per extra leg (0 = no extra legs)")
    ap.add_argument("--extra-warmup", type=int, default=1)
    ap.add_argument("--frames", type=int, default=100,
                    help="with config 3: median wall time of this many consecutive visualiser calls (calculatePSO, "
                         "N = 16384, 15 iterations), FAST and REFERENCE (0 = skip)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="gloo: rehearse the N>1 path with ranks sharing the visible GPUs (not a measurement)")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> None:
    """`--gpus N` from a plain `python bench.py`: start the N ranks as child
    processes (one per GPU) and exit with their status.  Nothing here touches
    the GPU, so the children start on a clean device; under torchrun
    (WORLD_SIZE set) the world must be the one --gpus names."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")
        return
    if args.gpus <= 1:
        return
    import torch  # device_count() does not initialise the GPU on this image

    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and ndev < args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {ndev} "
                 f"(--dist-backend gloo rehearses the N-rank path with ranks sharing the GPUs)")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve())]
    cmd += sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def valu_per_update(kernel: str):
    """VALU lane-instructions per particle-update of `kernel` (the solver's
    kernel name), from the committed rocprofv3 SQ_INSTS_VALU measurement
    (profiles/valu_per_update.json, tools/update_profiles.py), else None."""
    f = ROOT / "profiles" / "valu_per_update.json"
    if not f.exists():
        return None
    try:
        db = json.loads(f.read_text())
    except Exception:
        return None
    return db.get(kernel)


def _cpu_facts():
    """Host CPU model, CPUs in the machine, CPUs this process may run on, and
    the cgroup CPU quota (CPUs' worth of time, None if unlimited)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "cgroup_cpu_quota": quota}


def _cpu_sample(oracle, lib, wl, P, I, first, threads, seconds, max_batches, kw):
    """Batches of `threads` swarms of the workload (same targets and global
    seeds as the GPU run) until `seconds` have elapsed; returns (swarms, s)."""
    done, t0 = 0, time.perf_counter()
    for _ in range(max_batches):
        tg = wl.targets(first + done, threads)
        rng = oracle.init_generators(threads * P, (first + done) * P)
        oracle.solve_batch(wl.chain, tg, None, P, I, rng, threads=threads, lib=lib, **kw)
        done += threads
        if time.perf_counter() - t0 >= seconds:
            break
    return done, time.perf_counter() - t0


def cpu_baseline(seconds: float, threads: int, dh=None):
    """The CPU oracle (the reference algorithm restated in C, reference 4x4 FK
    order, -ffp-contract=off) built -O3 -march=native on this host, OpenMP over
    swarms, on bounded samples of configs 3 and 5 (BASELINE.md
    §4): every CPU of the affinity mask, and one thread."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    import ikpso

    facts = _cpu_facts()
    # every CPU of the affinity mask; where a cgroup quota grants fewer CPUs' worth of time, also that many
    # threads (oversubscribed threads only contend) -- the faster of the two is the baseline
    counts = [threads] if threads else sorted({facts["affinity_cpus"],
                                               min(facts["affinity_cpus"],
                                                   int(facts["cgroup_cpu_quota"] or facts["affinity_cpus"]))})
    build = "-O3 -march=native -ffp-contract=off -fopenmp"
    try:
        lib = oracle.load_native()
    except Exception as e:  # no compiler on this host: the prebuilt -O2 build
        lib, build = oracle.load(), f"-O2 -ffp-contract=off -fopenmp (native build failed: {type(e).__name__})"
    w3 = ikpso.workload(3)
    P, I = w3.particles, w3.iterations
    runs = {}
    for n in counts:
        done, el = _cpu_sample(oracle, lib, w3, P, I, 0, n, seconds, 64, {})
        runs[n] = (done * P * I / el, done, el)
    threads = max(runs, key=lambda n: runs[n][0])
    ups, done, el = runs[threads]
    d1, e1 = _cpu_sample(oracle, lib, w3, P, I, done, 1, 0.0, 1, {})  # one swarm, one thread
    # config 5: 20-joint chain, 4096 particles, penalty; a bounded number of iterations (the cost per
    # particle-update does not depend on I)
    w5 = ikpso.workload(5)
    I5 = 10
    kw5 = {"limit_weight": w5.limit_weight, "soft_lo": w5.soft_lo, "soft_hi": w5.soft_hi}
    d5, e5 = _cpu_sample(oracle, lib, w5, w5.particles, I5, 0, threads, seconds / 2, 16, kw5)
    dhres = None
    if dh is not None:  # the DH workload itself (axis mask as the GPU run; the oracle has one FK form)
        kwd = {"axis_mask": dh.axis_mask, "angle_weight": dh.fit.angle_weight}
        dd, ed = _cpu_sample(oracle, lib, dh, dh.particles, 50, 0, threads, seconds / 2, 16, kwd)
        dhres = {"value": dd * dh.particles * 50 / ed, "unit": "particle-updates/s", "cores": threads,
                 "sample": f"{dd} swarms x {dh.particles} particles x 50 iterations of {dh.name}, {ed:.1f} s"}
    return {"value": ups, "unit": "particle-updates/s", "cores": threads, "kind": "port", "arith": "reference",
            "dh": dhres,
            "solves_per_s": done / el, "value_1thread": d1 * P * I / e1, "build": build, **facts,
            "by_threads": {str(n): round(v[0]) for n, v in runs.items()},
            "sample": f"{done} swarms x {P} particles x {I} iterations of config 3 (same targets/seeds), "
                      f"OpenMP over swarms on {threads} threads, {el:.1f} s; 1 thread: 1 swarm, {e1:.1f} s",
            "config5": {"value": d5 * w5.particles * I5 / e5, "unit": "particle-updates/s", "cores": threads,
                        "sample": f"{d5} swarms x {w5.particles} particles x {I5} iterations of config 5, "
                                  f"{e5:.1f} s"}}


def timed_leg(ctx, wl, Bl, P, I, steps, warmup, arith="fast", kernel="auto", colliders=None):
    """One workload timed the driver's way on every rank: W untimed steps, then
    K steps between barrier + synchronize on both sides, max over ranks.  A step
    = one batch of Bl swarms per rank (ONE solver launch) + the all-gather of
    the per-swarm results + the copy to the host.  Returns the solver too (the
    caller closes it) and the row count the all-gather returned (checked against
    the swarms of all ranks)."""
    torch, dist, ikpso, idist, dev, world, rank = (ctx[k] for k in
                                                   ("torch", "dist", "ikpso", "idist", "dev", "world", "rank"))
    import numpy as np

    total, first = Bl * world, rank * Bl
    targets = torch.from_numpy(wl.targets(first, Bl)).to(dev)
    solver = ikpso.BatchSolver(wl.chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), fit=wl.fit, arith=arith,
                               limit_weight=wl.limit_weight, soft_lo=wl.soft_lo, soft_hi=wl.soft_hi,
                               kernel=kernel, axis_mask=wl.axis_mask, fold=wl.fold, colliders=colliders)
    solver.seed(Bl, seed_base=0, first_swarm=first)
    D = solver.dof
    out = (torch.empty((Bl, D), device=dev), torch.empty((Bl,), device=dev), torch.empty((Bl,), device=dev))
    host = torch.empty((total, D + 2), dtype=torch.float32, pin_memory=True)
    gathered = []

    def step(evs=None):
        if evs is not None:
            evs[0].record()
        solver.solve(targets, iterations=I, out=out)
        if evs is not None:
            evs[1].record()
        rows = idist.pack_results(*out)
        if world > 1:
            rows = idist.gather_rows(rows, total, world)
        gathered[:] = [int(rows.shape[0])]
        host.copy_(rows, non_blocking=True)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for k in range(steps):
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cpu" if ctx["backend"] == "gloo" else dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    res = host.numpy()
    if gathered[0] != total:
        raise RuntimeError(f"all-gather returned {gathered[0]} rows, expected {total}")
    return {"elapsed": float(t[0]), "kern_ms": float(t[1]), "solver": solver, "D": D, "total": total,
            "gathered_rows": gathered[0],
            "targets": targets, "first": first, "finite": bool(np.isfinite(res).all()),
            "mean_fitness": float(res[:, D].mean()), "mean_residual": float(res[:, D + 1].mean())}


def frame_latency(ikpso, torch, np, arith: str, frames: int = 100):
    """The visualiser's own call (src/Main.cpp:17,130,222-227): calculatePSO through the
    reference-compatible entry point with N = 16384 particles and PSOConfig(0.5, 0.5, 1.25, 15),
    generator states carried across frames, each answer fed back as the next frame's start pose
    (FromCoords, then ToCUDA).  One warm-up call, then the wall time of `frames` consecutive calls
    (the call is synchronous on return, like the reference's)."""
    P, D = 16384, 21
    old = os.environ.get("IKPSO_ARITH")
    os.environ["IKPSO_ARITH"] = arith  # the compat entry has no mode argument
    try:
        scene = ikpso.reference_scene(reset=True)
        chain = scene.origin.to_cuda()
        parts = ikpso.particles_tensor(P, D)
        bests = torch.zeros(P, dtype=torch.float32, device="cuda")
        rng = ikpso.rng_tensor(P)
        if ikpso.init_generators(rng, P) != 0:
            raise RuntimeError("initGenerators failed")
        res = np.zeros(D, dtype=np.float32)
        ts = []
        for k in range(frames + 1):
            t0 = time.perf_counter()
            st = ikpso.calculate_pso(parts, None, bests, rng, P, chain, ikpso.MAIN_PSO, ikpso.MAIN_FITNESS, res)
            dt = time.perf_counter() - t0
            if st != 0:
                raise RuntimeError(f"calculatePSO returned {st}")
            if k:
                ts.append(dt)
            scene.origin.from_coords(res)
            chain = scene.origin.to_cuda()
    finally:
        if old is None:
            os.environ.pop("IKPSO_ARITH", None)
        else:
            os.environ["IKPSO_ARITH"] = old
    t = np.array(ts) * 1e3
    return {"frame_ms": round(float(np.median(t)), 4), "p10_ms": round(float(np.percentile(t, 10)), 4),
            "p90_ms": round(float(np.percentile(t, 90)), 4), "frames": frames, "warmup": 1,
            "particle_updates_per_s": P * ikpso.MAIN_PSO.iterations / (float(np.median(t)) / 1e3),
            "residual_after": round(float(scene.check_distance()), 5)}


def rank_records(dist, torch, world: int, rank: int, local: int, backend: str):
    """What the process group itself reports, and every rank's device, gathered to all ranks."""
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    rec = {"rank": rank, "local_rank": local, "host": socket.gethostname(), "pid": os.getpid(),
           "device": torch.cuda.current_device(), "name": props.name,
           "pci": "{:04x}:{:02x}:{:02x}".format(getattr(props, "pci_domain_id", 0) or 0,
                                                getattr(props, "pci_bus_id", 0) or 0,
                                                getattr(props, "pci_device_id", 0) or 0),
           "uuid": str(getattr(props, "uuid", "") or "")}
    if world == 1:
        return {"world_size": 1, "backend": None, "ranks": [rec]}
    recs = [None] * world
    dist.all_gather_object(recs, rec)
    return {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "ranks": recs}


def valu_roofline(kernel: str, ups_launch: float, kern_ms: float, lib_id: str, arith: str = "fast"):
    """VALU lane-instructions per update (rocprofv3 SQ_INSTS_VALU x 64 / updates, committed in
    profiles/valu_per_update.json) x the live update rate, against the chip's 78.6 T lane-instructions/s
    (256 CU x 4 SIMD x 32 lanes x 2.4 GHz: every wave64 VALU op at its 2-cycle full rate).  None for a kernel
    without committed counters (or a streaming one: HBM-bound, priced by the caller)."""
    # the counters are per (kernel, arithmetic): a REFERENCE build of a kernel has its own entry
    key = kernel if arith == "fast" else f"{kernel} [{arith}]"
    vpu = None if "streaming" in kernel else valu_per_update(key)
    if not vpu:
        return None, None
    kern_s = kern_ms / 1e3
    instr = vpu["valu_lane_instr_per_update"]
    ach = ups_launch * instr / kern_s / 1e12
    # Secondary views.  gfx950 issue costs are not uniform (tools/probes/valu_probe.hip,
    # profiles/r02/valu_issue_costs.txt): v_lshlrev, v_add3, v_cvt, v_med3/max3 ... occupy 4.1 cycles,
    # v_sin/v_cos 8.1; the issue model (tools/issue_model.py on the kernel's ISA) prices the hot loop
    # opcode by opcode -- a roof lowered to the kernel's own instruction mix, not the chip's.
    trans = vpu.get("trans_lane_instr_per_update") or 0.0
    model = vpu.get("issue_model")
    slots_simple = instr + 3.0 * trans
    slots = instr * model["mean_cycles_per_instr"] / 2.0 if model else None
    valu = {"achieved": round(ach, 2), "peak": round(VALU_PEAK_TINSTR, 1), "unit": "Tlane-instr/s",
            "frac": round(ach / VALU_PEAK_TINSTR, 4),
            "instr_per_update": instr, "trans_per_update": trans, "source": vpu.get("source"),
            "measured_on_build": vpu.get("build_id"), "stale": vpu.get("build_id") != lib_id,
            "frac_issue_model": round(ups_launch * slots / kern_s / 1e12 / VALU_PEAK_TINSTR, 4)
            if slots else None,
            "issue_slots_per_update": round(slots, 1) if slots else None, "issue_model": model,
            "frac_uniform_cost": round(ups_launch * slots_simple / kern_s / 1e12 / VALU_PEAK_TINSTR, 4),
            "note": "frac = SQ_INSTS_VALU lane-instructions per update x updates/s / 78.6 T (chip peak, "
                    "every op at full rate); frac_issue_model: the same time priced at each opcode's "
                    "measured gfx950 issue cost (4-cycle integer/convert/med3 forms, 8-cycle sin/cos) -- "
                    "the fraction of the SIMDs' issue cycles the kernel's own mix keeps busy; "
                    "frac_uniform_cost: transcendentals as 4 slots. stale: the counters were measured on "
                    "another build than the loaded library"}
    return vpu, valu


def collide_leg(ctx, steps, warmup, lib_id, plain_ms):
    """The collider term (src/kernel.cu:104-136): config 3's batch (4096 targets per GPU,
    1024 particles, 500 iterations) with the reference's initColliders boxes 0 and 3 (src/Main.cpp:537-559:
    unit cubes at (1,0,0) and (0,0,1), which leave the reset pose clear), and the same collider kernel with
    the boxes moved 1000 units away (every pair rejected by the sphere test: the term's cost without GJK)."""
    ikpso = ctx["ikpso"]
    wl = ikpso.workload(3)
    boxes = ikpso.init_colliders(4)[[0, 3]]
    far = boxes.copy()
    far["pos"] += 1000.0
    P, I, Bl = wl.particles, wl.iterations, wl.swarms
    r = timed_leg(ctx, wl, Bl, P, I, steps, warmup, colliders=boxes)
    # boxes out of reach: the host-side early-out drops the term (the plain kernel runs); kept on the
    # collider kernel with IKPSO_KEEP_FAR_COLLIDERS=1 (the term's cost without any GJK)
    rf = timed_leg(ctx, wl, Bl, P, I, 1, 1, colliders=far)
    os.environ["IKPSO_KEEP_FAR_COLLIDERS"] = "1"
    try:
        rk = timed_leg(ctx, wl, Bl, P, I, 1, 1, colliders=far)
    finally:
        os.environ.pop("IKPSO_KEEP_FAR_COLLIDERS", None)
    vpu, valu = valu_roofline(r["solver"].kernel + " [colliders]", Bl * P * I, r["kern_ms"], lib_id)
    hbm = None
    if vpu:  # the counter-measured HBM bytes per update: the near nodes' stored frames and node_collides' spills
        gbs = Bl * P * I * vpu["hbm_bytes_per_update"] / (r["kern_ms"] / 1e3) / 1e9
        hbm = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
               "bytes_per_update": vpu["hbm_bytes_per_update"],
               "note": "FETCH_SIZE/WRITE_SIZE of the collider kernel: scratch traffic -- the frames of the nodes "
                       "near a collider (64 B each, written in the FK pass, read by the GJK pass) and "
                       "node_collides' register spills"}
    st = ROOT / "profiles" / "r05" / "collide_stats.json"
    leg = {"workload": f"config 3 with initColliders boxes 0 and 3: {wl.description}; {P} particles, {I} iterations",
           "value": r["total"] * P * I * steps / r["elapsed"], "unit": "particle-updates/s",
           "solves_per_s": r["total"] * steps / r["elapsed"], "ms_per_step": 1e3 * r["elapsed"] / steps,
           "kernel_ms": round(r["kern_ms"], 3), "steps": steps, "warmup": warmup, "swarms_per_gpu": Bl,
           "total_swarms": r["total"], "dof": r["D"], "kernel": r["solver"].kernel,
           "kernel_ms_far_colliders": round(rf["kern_ms"], 3), "far_colliders_kernel": rf["solver"].kernel,
           "far_colliders_tested": rf["solver"].collider_count,
           "kernel_ms_far_colliders_kept": round(rk["kern_ms"], 3), "kernel_ms_no_colliders": round(plain_ms, 3),
           "roofline_frac": valu["frac"] if valu else None,
           "roofline_stale": valu["stale"] if valu else None,
           "roofline_hbm": hbm,
           "early_out": json.loads(st.read_text()) if st.exists() else None,
           "check": {"finite": r["finite"], "mean_fitness": r["mean_fitness"],
                     "mean_residual": r["mean_residual"]}}
    for x in (r, rf, rk):
        x["solver"].close()
    return leg


def extra_leg(ctx, name, steps, warmup, lib_id, cpu=None):
    """Another BASELINE line measured in the same run (every rank, same timing rules as the headline):
    4 = config 4's shard, 8192 targets per GPU (N = 8: the named 65536); 5 = config 5, its named 8192 targets
    over all GPUs; dh7 = the DH arm, 4096 targets per GPU."""
    ikpso, world = ctx["ikpso"], ctx["world"]
    wl = ikpso.workload(name)
    if name == "4":
        Bl, wname = 8192, "config 4 (8192 targets per GPU; 65536 at N = 8)"
    elif name == "5":
        Bl, wname = -(-wl.swarms // world), "config 5 (8192 targets over all GPUs)"
    else:
        Bl, wname = wl.swarms, f"{name} (4096 targets per GPU)"
    P, I = wl.particles, wl.iterations
    r = timed_leg(ctx, wl, Bl, P, I, steps, warmup)
    ups_launch = Bl * P * I
    _, valu = valu_roofline(r["solver"].kernel, ups_launch, r["kern_ms"], lib_id)
    leg = {"workload": f"{wname}: {wl.description}; {P} particles, {I} iterations",
           "value": r["total"] * P * I * steps / r["elapsed"], "unit": "particle-updates/s",
           "solves_per_s": r["total"] * steps / r["elapsed"], "ms_per_step": 1e3 * r["elapsed"] / steps,
           "kernel_ms": round(r["kern_ms"], 3), "steps": steps, "warmup": warmup, "swarms_per_gpu": Bl,
           "total_swarms": r["total"], "dof": r["D"], "kernel": r["solver"].kernel,
           "roofline_frac": valu["frac"] if valu else None,
           "roofline_frac_issue_model": valu["frac_issue_model"] if valu else None,
           "roofline_stale": valu["stale"] if valu else None,
           "check": {"finite": r["finite"], "mean_fitness": r["mean_fitness"], "mean_residual": r["mean_residual"]}}
    if cpu is not None:
        leg["cpu_baseline"] = cpu
    r["solver"].close()
    return leg


def summary(line: dict, value: float) -> dict:
    """Compact restatement of the line's figures (rounded), printed last."""
    r3 = lambda x: None if x is None else float(f"{x:.4g}")
    out = {"value": r3(value), "kernel_ms": line["roofline"].get("kernel_ms"),
           "roofline_frac": line["roofline"].get("frac"), "single_solve_ms": r3(line.get("single_solve_ms")),
           "single_solve_p10_ms": r3(line.get("single_solve_p10_ms"))}
    if line.get("frame"):
        out["frame_ms"] = {a: f["frame_ms"] for a, f in line["frame"].items()}
    if line.get("reference_arith"):
        ra = line["reference_arith"]
        out["reference_arith"] = {"value": r3(ra["value"]), "kernel_ms": ra["kernel_ms"],
                                  "roofline_frac": ra["roofline_frac"]}
    for name, leg in (line.get("legs") or {}).items():
        out[name] = {"value": r3(leg["value"]), "kernel_ms": leg["kernel_ms"], "roofline_frac": leg["roofline_frac"]}
        for k in ("kernel_ms_far_colliders", "kernel_ms_far_colliders_kept", "kernel_ms_no_colliders"):
            if k in leg:
                out[name][k] = leg[k]
    cpu = line.get("cpu_baseline")
    if cpu:
        out["cpu_baseline"] = {"value": r3(cpu["value"]), "cores": cpu["cores"], "kind": cpu["kind"],
                               "value_1thread": r3(cpu.get("value_1thread"))}
    return out


def main():
    args = parse()
    launch_ranks(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    import ikpso
    from ikpso import dist as idist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.dist_backend == "gloo":
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group("gloo")
    elif world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    group = rank_records(dist, torch, world, rank, local, args.dist_backend)
    ctx = {"torch": torch, "dist": dist, "ikpso": ikpso, "idist": idist, "dev": dev, "world": world,
           "rank": rank, "backend": args.dist_backend}

    wl = ikpso.workload(args.config)
    cfg = int(args.config) if args.config.isdigit() else args.config
    P = args.particles or wl.particles
    I = args.iterations or wl.iterations
    if args.swarms_per_gpu:
        Bl = args.swarms_per_gpu
    elif cfg == 3 or not isinstance(cfg, int):
        Bl = wl.swarms                      # weak scaling: 4096 per GPU
    else:
        Bl = -(-wl.swarms // world)         # configs 4/5: the named total over all GPUs

    # the bounded CPU baseline runs before the GPU legs, on rank 0 at every N (north_star: the CPU path
    # "alongside" at 1, 2, 4 and 8 GPUs); the other ranks wait for it at a barrier
    cpu = None
    if rank == 0 and args.cpu_seconds > 0 and cfg in (3, 5, "dh7", "dh7-nofold", "dh7-locked"):
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_threads, dh=wl if isinstance(cfg, str) else None)
        if cfg == 5:  # the config-5 figure is this line's baseline
            cpu = dict(cpu, value=cpu["config5"]["value"], sample=cpu["config5"]["sample"])
        if isinstance(cfg, str):  # the DH arm's own figure
            cpu = dict(cpu, value=cpu["dh"]["value"], sample=cpu["dh"]["sample"])
        if world > 1:
            cpu["note"] = f"rank 0's host cores, timed before the GPU legs while ranks 1..{world - 1} waited"
    if world > 1:
        dist.barrier()

    colliders = None
    if args.colliders != "none":
        colliders = ikpso.init_colliders(4)
        if args.colliders == "init03":
            colliders = colliders[[0, 3]]
        elif args.colliders == "far4":
            colliders["pos"] += 1000.0
    main_leg = timed_leg(ctx, wl, Bl, P, I, args.steps, args.warmup, args.arith, args.kernel, colliders=colliders)
    solver, D, total = main_leg["solver"], main_leg["D"], main_leg["total"]
    elapsed, kern_ms = main_leg["elapsed"], main_leg["kern_ms"]
    targets, first = main_leg["targets"], main_leg["first"]
    ups_step = total * P * I
    value = ups_step * args.steps / elapsed

    single_ms = single_p10 = None
    if rank == 0 and cfg != 5 and colliders is None:
        s2 = ikpso.BatchSolver(wl.chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), fit=wl.fit, arith=args.arith,
                               axis_mask=wl.axis_mask, fold=wl.fold)
        s2.seed(1)
        tg1 = targets[:1].contiguous()
        out1 = (torch.empty((1, D), device=dev), torch.empty((1,), device=dev), torch.empty((1,), device=dev))
        ans = torch.empty((1, D), dtype=torch.float32, pin_memory=True)  # the answer's host buffer, allocated once
        s2.solve(tg1, iterations=I, out=out1)
        torch.cuda.synchronize()
        # wall time of one solve to its answer on the host: the median of 50 (round 5 took 5, whose median
        # moved 1.34 -> 1.46 ms between boxes while the kernel itself did not: profiles/r06/variant_timings/
        # var_c2_r4_vs_cur.txt, round 4's build and this one interleaved, 1.375 vs 1.373 ms)
        ts = []
        stream = torch.cuda.current_stream()
        for _ in range(50):
            a = time.perf_counter()
            s2.solve(tg1, iterations=I, out=out1)
            ans.copy_(out1[0], non_blocking=True)
            stream.synchronize()
            ts.append(time.perf_counter() - a)
        single_ms = 1e3 * float(np.median(ts))
        single_p10 = 1e3 * float(np.percentile(ts, 10))
        s2.close()

    # the REFERENCE-arithmetic (bit-identical to the oracle) throughput of the same workload, driver-measured
    reference_arith = None
    if rank == 0 and args.arith == "fast" and args.reference_steps > 0 and cfg in (3, 4) and colliders is None:
        sr = ikpso.BatchSolver(wl.chain, P, pso=ikpso.PSOConfig(0.5, 0.5, 1.25, I), fit=wl.fit, arith="reference",
                               kernel=args.kernel)
        sr.seed(Bl, seed_base=0, first_swarm=first)
        out_r = (torch.empty((Bl, D), device=dev), torch.empty((Bl,), device=dev), torch.empty((Bl,), device=dev))
        sr.solve(targets, iterations=I, out=out_r)
        torch.cuda.synchronize()
        evr = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.reference_steps)]
        tr = time.perf_counter()
        for a, b in evr:
            a.record()
            sr.solve(targets, iterations=I, out=out_r)
            b.record()
        torch.cuda.synchronize()
        el_r = time.perf_counter() - tr
        rk = sr.kernel
        _, rvalu = valu_roofline(rk, Bl * P * I, float(np.mean([a.elapsed_time(b) for a, b in evr])),
                                 ikpso.build_id(), arith="reference")
        reference_arith = {"value": Bl * P * I * args.reference_steps / el_r, "unit": "particle-updates/s",
                           "kernel_ms": round(float(np.mean([a.elapsed_time(b) for a, b in evr])), 3),
                           "steps": args.reference_steps, "warmup": 1, "kernel": rk,
                           "roofline_frac": rvalu["frac"] if rvalu else None,
                           "roofline_stale": rvalu["stale"] if rvalu else None,
                           "swarms": Bl, "check_finite": bool(torch.isfinite(out_r[1]).all()),
                           "note": "REFERENCE arithmetic: the reference's 4x4 operation order, no FMA contraction, "
                                   "correctly rounded sin/cos -- bit-identical to the CPU oracle "
                                   "(tests/test_gpu_parity.py) and, through it, to the reference's recorded CUDA "
                                   "run (tests/test_gpu_trajectory.py); same workload, rank 0"}
        sr.close()

    # the visualiser's own per-frame call (N = 16384, 15 iterations), both arithmetic modes
    frame = None
    if rank == 0 and cfg == 3 and args.frames > 0 and colliders is None:
        frame = {a: frame_latency(ikpso, torch, np, a, args.frames) for a in ("fast", "reference")}

    lib_id = ikpso.build_id()
    # the other BASELINE lines, same run and timing rules (every rank): config 4's per-GPU shard, config 5 at
    # its named size, the DH arm -- after the headline legs so the GPU stays busy to the end of the run
    legs = {}
    if cfg == 3 and args.extra_steps > 0 and colliders is None:
        for name in args.extra_legs.split(","):
            name = name.strip()
            if name == "collide":
                legs[name] = collide_leg(ctx, args.extra_steps, args.extra_warmup, lib_id, kern_ms)
            elif name:
                c5 = cpu.get("config5") if (cpu and name == "5") else None
                legs["config" + name if name.isdigit() else name] = extra_leg(
                    ctx, name, args.extra_steps, args.extra_warmup, lib_id, c5)

    if rank == 0:
        ups_launch = Bl * P * I
        kern_s = kern_ms / 1e3
        alg_bytes = 20 * D + 8
        alg_gbs = ups_launch * alg_bytes / kern_s / 1e9
        streaming = "streaming" in solver.kernel
        vpu, valu = valu_roofline(solver.kernel + (" [colliders]" if colliders is not None else ""), ups_launch,
                                  kern_ms, lib_id, args.arith)
        # the streaming kernels move x/v/pbest through HBM (HBM-bound); an on-chip kernel without a committed
        # PMC profile is reported unmeasured rather than against the HBM formulation it does not use
        on_chip_unmeasured = not streaming and not valu
        roofline = {
            "bound": "valu" if valu or on_chip_unmeasured else "hbm",
            "achieved": valu["achieved"] if valu else (None if on_chip_unmeasured else round(alg_gbs, 1)),
            "peak": valu["peak"] if valu else (round(VALU_PEAK_TINSTR, 1) if on_chip_unmeasured else HBM_PEAK_GBS),
            "unit": valu["unit"] if valu else ("Tlane-slot/s" if on_chip_unmeasured else "GB/s"),
            "frac": valu["frac"] if valu else (None if on_chip_unmeasured else round(alg_gbs / HBM_PEAK_GBS, 4)),
            "traffic": round(vpu["hbm_bytes_per_update"] * ups_launch) if vpu else None,
            "kernel": solver.kernel + (" (I+2 launches per batch)" if streaming else " (one launch = one batch)"),
            "stale": bool(valu and valu["stale"]),
            "kernel_ms": round(kern_ms, 3),
            "hbm_measured": None if not vpu else {
                "achieved": round(ups_launch * vpu["hbm_bytes_per_update"] / kern_s / 1e9, 2),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ups_launch * vpu["hbm_bytes_per_update"] / kern_s / 1e9 / HBM_PEAK_GBS, 6),
                "bytes_per_update": vpu["hbm_bytes_per_update"],
                "note": "counter-measured HBM bytes per particle-update ((2*FETCH_SIZE + WRITE_SIZE) of the "
                        "kernel's dispatch, profiles/valu_per_update.json) x the live update rate: the swarm "
                        "state stays on chip, HBM carries only generator states, inputs and results",
            },
            "hbm_algorithmic": {
                "achieved": round(alg_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(alg_gbs / HBM_PEAK_GBS, 4),
                "bytes_per_update": alg_bytes,
                "note": "SURVEY §8(d) north-star formulation (x/v/pbest streamed through HBM every iteration); "
                        "this kernel keeps them on chip, so the figure can exceed 1 and the binding roof is VALU",
            },
        }
        metric = {5: "PSO particle-updates/sec + IK solves/sec, 20-DOF 4096-particle swarm (config 5)"}.get(
            cfg, "PSO particle-updates/sec + IK solves/sec, 7-DOF 1024-particle swarm")
        if isinstance(cfg, str):
            metric += f" ({cfg}: 7-joint DH arm, D = {D})"
        line = {
            "metric": metric,
            "value": value,
            "unit": "particle-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": {2: "the reference scene's reset targets (src/Main.cpp:334-336)",
                     5: "synthetic (seeded targets uniform in a radius-2..4 shell)"}.get(
                cfg, "synthetic (seeded reachable targets: the arm's tool positions at seeded joint angles)"
                if isinstance(cfg, str) else "synthetic (seeded targets: reset targets + U[-0.25,0.25]^3 per effector)"),
            "config": {
                "workload": f"{wl.name}: {wl.description}; {P} particles, {I} PSO iterations, "
                            f"{Bl} targets per GPU ({total} total)",
                "swarms_per_gpu": Bl, "total_swarms": total, "particles": P, "iterations": I, "dof": D,
                "parallelism": f"dp{world} (swarm shards) + {'RCCL' if args.dist_backend == 'nccl' else 'gloo (rehearsal)'}"
                               f" all-gather of results; process group: world_size {group['world_size']}, backend "
                               f"{group['backend']}, {len({r['pci'] + r['host'] for r in group['ranks']})} distinct "
                               f"devices, {main_leg['gathered_rows']} rows gathered" if world > 1
                else "1 GPU",
                "process_group": dict(group, gathered_rows=main_leg["gathered_rows"]),
                "arith": args.arith,
                "colliders": args.colliders,
            },
            "solves_per_s": total * args.steps / elapsed,
            "single_solve_ms": single_ms,
            "single_solve_p10_ms": single_p10,
            "roofline": roofline,
            "reference_arith": reference_arith,
            "legs": legs or None,
            "frame": frame,
            "cpu_baseline": cpu,
            "speedup_vs_cpu": None if not cpu else {
                "fast": round(value / cpu["value"], 1),
                "like_for_like": round(reference_arith["value"] / cpu["value"], 1) if reference_arith else None,
                "note": "fast: the headline (FAST arithmetic) over the CPU oracle (REFERENCE arithmetic); "
                        "like_for_like: the GPU's REFERENCE-arithmetic leg (bit-identical results) over the same "
                        "CPU oracle"},
            "build_id": lib_id,
            "check": {"finite": main_leg["finite"], "mean_fitness": main_leg["mean_fitness"],
                      "mean_residual": main_leg["mean_residual"]},
            "parity": f"{args.arith.upper()} arithmetic. REFERENCE mode is bit-identical to the CPU oracle "
                      "(tests/test_gpu_parity.py), and the oracle and the REFERENCE kernels replay the reference's "
                      "own recorded CUDA run (results.xlsx DEGREES_3: every case start and 506 of 661 frames within "
                      "1e-5 rad, tests/test_trajectory.py, tests/test_gpu_trajectory.py) -- which pins cuRAND's "
                      "seeding and uniform mapping, the draw order, update, clamp, FK, fitness and argmin against "
                      "the reference itself. FAST (benchmarked) holds FK |dp| <= 2e-5, tier A |dtheta| <= 1e-4 "
                      "(also against the recording), tier B per-swarm bounds (tests/test_gpu_parity.py).",
        }
        if valu:
            line["roofline"]["valu"] = valu
        elif on_chip_unmeasured:
            line["roofline"]["note"] = (f"no committed rocprofv3 PMC profile of {solver.kernel} "
                                        "(profiles/valu_per_update.json): VALU fraction unmeasured for this line")
        if cfg == 2:
            line["roofline"]["note"] = ("config 2 is one swarm on 4 of 256 CUs: latency-bound (SURVEY 8(d)), "
                                        "the chip-wide fraction is not a kernel-quality figure")
        # the line's last key: the other BASELINE lines in a few hundred bytes, so a reader that keeps only the
        # tail of a long line (the driver's record) still has config 2's latency, the frame and every leg
        line["summary"] = summary(line, value)
        print(json.dumps(line), flush=True)
    solver.close()
    if world > 1:
        dist.barrier()  # rank 0's extra timing runs finish before any rank tears down
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
