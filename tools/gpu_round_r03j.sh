#!/bin/bash
# Round 3: generator-split latency variant with 128- vs 256-particle chunks (variants/lat_*.so),
# then the full GPU suite and the config-2 bench line on the shipped build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== variants B=1"
IKPSO_ALLOW_STALE=1 timeout -k 10 300 python -u tools/variant_bench.py variants/lat_*.so --config 3 --swarms 1 --rounds 7 \
  > gpurun_out/var_lat1.txt 2>&1 || exit 3
echo "== variants B=8"
IKPSO_ALLOW_STALE=1 timeout -k 10 300 python -u tools/variant_bench.py variants/lat_*.so --config 3 --swarms 8 --rounds 5 \
  > gpurun_out/var_lat8.txt 2>&1 || exit 4
echo "== all tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit 6
echo "== bench config 2"
timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 3 --cpu-seconds 3 > gpurun_out/bench_config2.json \
  2> gpurun_out/bench_config2.err || exit 5
echo "== frame"; timeout -k 10 300 python tools/frame_bench.py > gpurun_out/frame.log 2>&1 || exit 7
echo ALL_DONE
