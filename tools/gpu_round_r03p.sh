#!/bin/bash
# Round 3: wide latency groups with linear (cross-XCD) membership -- the visualiser frame, then every GPU test
# and the config-2 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== frame"; timeout -k 10 300 python tools/frame_bench.py > gpurun_out/frame.log 2>&1 || exit 5
grep -v amdgpu gpurun_out/frame.log
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
echo "== config 2"; timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 3 --cpu-seconds 3 > gpurun_out/bench_config2.json 2> gpurun_out/bench_config2.err || exit 4
echo ALL_DONE
