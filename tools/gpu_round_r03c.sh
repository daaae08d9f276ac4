#!/bin/bash
# Round 3, revolution-space kernels: every GPU test, smoke, the three bench lines, then config-5 variants.
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
echo ROUND_DONE
[ -n "$1" ] && { bash tools/gpu_var.sh "$@" || exit 7; }
echo ALL_DONE
