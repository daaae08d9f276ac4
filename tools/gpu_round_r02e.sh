#!/bin/bash
# Round-2 GPU session for the tip-backward build: every GPU test, smoke, the
# config-5 line and the default bench line, then the previous build's config-5
# kernel (variants/c5_L4.so) against this one, interleaved in one process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit 3
echo "== bench5"; timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_config5.json 2> gpurun_out/bench5.err || exit 5
echo "== dh7"; timeout -k 10 300 python bench.py --config dh7 --steps 5 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_dh7.json 2> gpurun_out/bench_dh7.err || exit 6
echo "== variants c5"
timeout -k 10 400 python tools/variant_bench.py variants/c5_L4.so inverse-kinematics-pso-research_amd/ikpso/_lib/libikpso.so \
    --config 5 --swarms 2048 --iters 100 --rounds 3 > gpurun_out/var_c5.txt 2>&1 || exit 9
echo ROUND_DONE
