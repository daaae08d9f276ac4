#!/bin/bash
# Round-3 first GPU session: every GPU test (new: config 5 at its own size, the
# RCCL world-1 branch, the wide-angle routing, the families' FAST agreement),
# smoke, the default / config-5 / dh7 bench lines (plain VALU fraction, build id,
# REFERENCE-arithmetic leg), the extended trig probe, then config 3's PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.txt 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit 3
echo "== bench"; timeout -k 10 400 python bench.py > gpurun_out/bench_config3.json 2> gpurun_out/bench_config3.err || exit 4
echo "== bench5"; timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_config5.json 2> gpurun_out/bench5.err || exit 5
echo "== dh7"; timeout -k 10 300 python bench.py --config dh7 --steps 5 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_dh7.json 2> gpurun_out/bench_dh7.err || exit 6
echo "== trig probe"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinverse-kinematics-pso-research_amd/csrc -Iinclude tools/probes/trig_probe.hip -o /tmp/trig_probe && \
  timeout -k 10 120 /tmp/trig_probe > gpurun_out/trig_probe.txt 2>&1 || exit 7
echo ROUND_DONE
echo "== PMC config 3"
PROF_NAME=c3 PROF_ARGS="--swarms-per-gpu 2048 --steps 2 --warmup 1 --cpu-seconds 0 --reference-steps 0" bash tools/gpu_profile.sh || exit 8
echo PMC_DONE
