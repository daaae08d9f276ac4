#!/bin/bash
# Round 3, generator-split latency variant: the GPU tests of the kernels it replaces
# (AUTO on few swarms), then config-2 variant timings (split vs unsplit, the
# generator's work split between step and hand-off, timing builds), then the full suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== latency-variant tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coop.py -m gpu -v -x -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_lat.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_lat.txt
[ $rc -eq 0 ] || exit 2
echo "== variants B=1"
IKPSO_ALLOW_STALE=1 timeout -k 10 300 python -u tools/variant_bench.py variants/lat_*.so --config 3 --swarms 1 --rounds 7 \
  > gpurun_out/var_lat1.txt 2>&1 || exit 3
echo "== variants B=16"
IKPSO_ALLOW_STALE=1 timeout -k 10 300 python -u tools/variant_bench.py variants/lat_*.so --config 3 --swarms 16 --rounds 5 \
  > gpurun_out/var_lat16.txt 2>&1 || exit 4
echo "== bench config 2"
timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 3 --cpu-seconds 3 > gpurun_out/bench_config2.json \
  2> gpurun_out/bench_config2.err || exit 5
echo "== all tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit 6
echo ALL_DONE
