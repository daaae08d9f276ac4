#!/bin/bash
# Round 3: the coop tests (visualiser-size latency groups), the visualiser frame and the examples.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_examples.py -m gpu -v -x -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_coop.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_coop.txt
[ $rc -eq 0 ] || exit 2
echo "== frame"; timeout -k 10 300 python tools/frame_bench.py > gpurun_out/frame.log 2>&1 || exit 5
grep -v amdgpu gpurun_out/frame.log
echo ALL_DONE
