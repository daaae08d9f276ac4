#!/bin/bash
# Round 3: prescaled draws in the generator-split latency variant (variants/lat_*.so) + the latency-variant
# tests (parity, DH, coop) on the shipped build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== variants B=1"
IKPSO_ALLOW_STALE=1 timeout -k 10 300 python -u tools/variant_bench.py variants/lat_*.so --config 3 --swarms 1 --rounds 7 \
  > gpurun_out/var_lat1.txt 2>&1 || exit 3
echo "== latency tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dh.py tests/test_gpu_coop.py -m gpu -v -x \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_lat.txt 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_lat.txt; [ $rc -eq 0 ] || exit 2
echo ALL_DONE
