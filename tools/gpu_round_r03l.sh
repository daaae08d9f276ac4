#!/bin/bash
# Round 3 verification of the shipped build (generator-split latency variant): every GPU test, smoke, the
# default / config-5 / dh7 / config-2 bench lines, the visualiser frame, the rocprofv3 kernel trace of the
# default bench command, then the PMC passes of the three benchmarked kernels (stamped with the build id).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit 3
echo "== bench"; timeout -k 10 400 python bench.py > gpurun_out/bench_config3.json 2> gpurun_out/bench_config3.err || exit 4
echo "== bench5"; timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_config5.json 2> gpurun_out/bench5.err || exit 5
echo "== dh7"; timeout -k 10 300 python bench.py --config dh7 --steps 5 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_dh7.json 2> gpurun_out/bench_dh7.err || exit 6
echo "== config 2"; timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 3 --cpu-seconds 3 > gpurun_out/bench_config2.json 2> gpurun_out/bench_config2.err || exit 7
echo "== frame"; timeout -k 10 300 python tools/frame_bench.py > gpurun_out/frame.log 2>&1 || exit 8
echo "== rocprof default bench"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- \
    python3 bench.py > gpurun_out/bench_under_rocprof.json 2> gpurun_out/bench_under_rocprof.err || exit 9
echo "== rocprof config 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_config2 -o run --output-format csv -- \
    python3 bench.py --config 2 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/bench2_under_rocprof.json 2> gpurun_out/bench2_under_rocprof.err || exit 10
echo ROUND_DONE
PROF_NAME=c3 PROF_ARGS="--swarms-per-gpu 2048 --steps 2 --warmup 1 --cpu-seconds 0 --reference-steps 0" bash tools/gpu_profile.sh || exit 11
PROF_NAME=c5 PROF_ARGS="--config 5 --swarms-per-gpu 2048 --iterations 100 --steps 2 --warmup 1 --cpu-seconds 0" bash tools/gpu_profile.sh || exit 12
PROF_NAME=dh7 PROF_ARGS="--config dh7 --swarms-per-gpu 2048 --steps 2 --warmup 1 --cpu-seconds 0" bash tools/gpu_profile.sh || exit 13
echo PMC_DONE
