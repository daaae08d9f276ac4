#!/bin/bash
# Round 3: the poll-first exchange (short chains) -- every GPU test, smoke, config-2 and default bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit 3
echo "== config 2"; timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 3 --cpu-seconds 3 > gpurun_out/bench_config2.json 2> gpurun_out/bench_config2.err || exit 4
echo "== frame"; timeout -k 10 300 python tools/frame_bench.py > gpurun_out/frame.log 2>&1 || exit 5
echo ALL_DONE
