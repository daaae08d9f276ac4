#!/bin/bash
# One GPU session on the gpurun box, as a list of stages run in order:
#
#   tools/gpu_session.sh STAGE [STAGE ...]
#
#   tests        every -m gpu test (IKPSO_REPORT_DIR=gpurun_out/reports: the tier-B and
#                trajectory distributions); TESTS="<paths/-k ...>" narrows it
#   smoke        __graft_entry__.smoke()
#   bench        the default bench line (BENCH_ARGS adds flags) -> gpurun_out/bench.json
#   bench:<cfg>  bench.py --config <cfg> (3 steps) -> gpurun_out/bench_<cfg>.json
#   gloo2        the N = 2 path rehearsed on the one GPU (two ranks over gloo sharing it; not a
#                measurement): the default line with its config-4 leg at 2 x 8192 targets and
#                rank 0's CPU baseline
#   rocprof      rocprofv3 kernel trace of the default bench command (its average kernel
#                duration must agree with the line's HIP-event kernel_ms)
#   profile:<n>  kernel trace + PMC passes (tools/gpu_profile.sh) of workload n in
#                {c3, c5, dh7, c3ref, collide}: the counters bench.py's roofline reads
#   hwcomp       v_sin/v_cos amplitude error on the tier-B answers' angles + the link-length
#                compensation experiment (tools/hwtrig_comp.py; HWCOMP_EPS = eps list)
#   collconsist  FAST collider solve vs evaluate kernel (tools/collide_consistency.py; VLIBS = variants)
#   collcmp      collider kernel ms, boxes near / far (tools/collide_cmp.sh; VARIANTS = product coll_vN ...)
#   frame        the visualiser frame latency (tools/frame_bench.py)
#   collstats    collider-term counters (tools/collide_stats.py) with vlib6/collide_stats.so
#   frametrace   rocprofv3 kernel trace of the same (what device work one frame issues)
#   var:<out>    interleaved variant timing (tools/gpu_var.sh; VAR_ARGS = "CONFIG SWARMS ITERS LIB...")
#   asan         host-code ASan/UBSan run (tools/asan_check.sh)
#
# Every GPU step has its own time limit; a crash, abort or timeout (anything but a
# plain test failure) ends the session so nothing else touches the GPU after a fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "   rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400
  return $rc
}
for s in "$@"; do
  case $s in
    tests)
      IKPSO_REPORT_DIR=gpurun_out/reports step gpu_tests 1100 python -u -m pytest ${TESTS:-tests} -m gpu -v -x -s \
        -p no:cacheprovider --timeout 300 --timeout-method thread
      rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 2 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 3 ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} || exit 4; tail -1 gpurun_out/bench.log > gpurun_out/bench.json ;;
    bench:*)
      c=${s#bench:}
      step "bench_$c" 600 python bench.py --config "$c" --steps 3 --warmup 1 --cpu-seconds 4 || exit 4
      tail -1 "gpurun_out/bench_$c.log" > "gpurun_out/bench_$c.json" ;;
    gloo2)
      step gloo2 600 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --cpu-seconds 4 || exit 4
      grep '^{' gpurun_out/gloo2.log | tail -1 > gpurun_out/bench_gloo2.json ;;
    rocprof)
      step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- \
        python3 bench.py ${BENCH_ARGS:-} || exit 5 ;;
    profile:c3) PROF_NAME=c3 PROF_ARGS="--swarms-per-gpu 2048 --steps 2 --warmup 1 --cpu-seconds 0 --extra-steps 0" \
                bash tools/gpu_profile.sh || exit 6 ;;
    profile:c3ref) PROF_NAME=c3ref PROF_ARGS="--arith reference --swarms-per-gpu 2048 --iterations 200 --steps 1 \
                   --warmup 1 --cpu-seconds 0 --reference-steps 0 --extra-steps 0" bash tools/gpu_profile.sh || exit 6 ;;
    profile:dh7) PROF_NAME=dh7 PROF_ARGS="--config dh7 --swarms-per-gpu 2048 --steps 2 --warmup 1 --cpu-seconds 0" \
                 bash tools/gpu_profile.sh || exit 6 ;;
    profile:collide) PROF_NAME=collide PROF_ARGS="--colliders init03 --swarms-per-gpu 2048 --steps 2 --warmup 1 \
                     --cpu-seconds 0" bash tools/gpu_profile.sh || exit 6 ;;
    profile:c5) PROF_NAME=c5 PROF_ARGS="--config 5 --swarms-per-gpu 2048 --iterations 100 --steps 1 --warmup 1 \
                --cpu-seconds 0" bash tools/gpu_profile.sh || exit 6 ;;
    hwcomp)  # the transcendental unit's amplitude error on the fixtures' answer angles, and the link-length
             # compensation experiment (tools/hwtrig_comp.py)
      python -c "import numpy as np; [np.load(f'tests/golden/tierb_config{c}.npz')['ref_angles'].astype(np.float32).tofile(f'gpurun_out/c{c}_angles.f32') for c in (3, 5)]" || exit 11
      step hwprobe 120 tools/probes/hwtrig_bias gpurun_out/c5_angles.f32 gpurun_out/c3_angles.f32 || exit 11
      step hwcomp 600 python -u tools/hwtrig_comp.py ${HWCOMP_EPS:-} || exit 11 ;;
    collconsist)  # FAST collider solve vs evaluate kernel on the solve's answers (product, then VLIBS variants)
      [ "${PRODUCT:-1}" = 0 ] || step collconsist_product 300 python -u tools/collide_consistency.py || exit 12
      for v in ${VLIBS:-}; do
        IKPSO_LIB=vlib6/$v.so IKPSO_ALLOW_STALE=1 step "collconsist_$v" 300 python -u tools/collide_consistency.py || exit 12
      done ;;
    collcmp) step collcmp 900 env VARIANTS="${VARIANTS:-product}" bash tools/collide_cmp.sh || exit 13 ;;
    frame) step frame 300 python tools/frame_bench.py || exit 7 ;;
    collstats) [ -f vlib6/collide_stats.so ] || { echo "no vlib6/collide_stats.so"; exit 10; }
      for sc in init03 far4 init4; do
        IKPSO_LIB=vlib6/collide_stats.so IKPSO_ALLOW_STALE=1 step "collstats_$sc" 300 \
          python tools/collide_stats.py ${COLL_SWARMS:-1024} 500 $sc "gpurun_out/collide_stats_$sc.json" || exit 10
      done ;;
    frametrace)
      step frametrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_frame -o run --output-format csv -- \
        python3 tools/frame_bench.py || exit 7 ;;
    var:*) bash tools/gpu_var.sh "${s#var:}" $VAR_ARGS || exit 8 ;;
    asan) step asan 600 bash tools/asan_check.sh run || exit 9 ;;
    *) echo "unknown stage $s"; exit 64 ;;
  esac
done
echo SESSION_DONE
