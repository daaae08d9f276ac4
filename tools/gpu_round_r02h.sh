#!/bin/bash
# Round-2 final GPU session (2-level wave priority in the 4-wave pipelined step):
# every GPU test, smoke, the default / config-5 / dh7 bench lines and the
# rocprofv3 kernel trace of the default bench command, then config 3's PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit 3
echo "== bench"; timeout -k 10 300 python bench.py > gpurun_out/bench_config3.json 2> gpurun_out/bench_config3.err || exit 4
echo "== rocprof default bench"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- \
    python3 bench.py > gpurun_out/bench_under_rocprof.json 2> gpurun_out/bench_under_rocprof.err || exit 7
echo "== bench5"; timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_config5.json 2> gpurun_out/bench5.err || exit 5
echo "== dh7"; timeout -k 10 300 python bench.py --config dh7 --steps 5 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_dh7.json 2> gpurun_out/bench_dh7.err || exit 6
echo ROUND_DONE
echo "== PMC config 3"
PROF_NAME=c3 PROF_ARGS="--swarms-per-gpu 2048 --steps 2 --warmup 1 --cpu-seconds 0" bash tools/gpu_profile.sh || exit 8
echo PMC_DONE
