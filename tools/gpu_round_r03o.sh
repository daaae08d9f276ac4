#!/bin/bash
# Round 3: compat-path host overhead (host inputs copied on the CPU, one synchronisation for the error flag and
# the answer): the compat/coop/parity GPU tests and the visualiser frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== frame"; timeout -k 10 300 python tools/frame_bench.py > gpurun_out/frame.log 2>&1 || exit 5
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
echo ALL_DONE
