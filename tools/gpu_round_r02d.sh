#!/bin/bash
# Round-2 GPU session for the wave-priority build: every GPU test, smoke, the
# default bench line, config 5 and the folded DH arm, the rocprofv3 kernel trace
# of the default bench command, then config 5's PMC passes (tools/gpu_profile.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit 3
echo "== bench"; timeout -k 10 300 python bench.py > gpurun_out/bench_config3.json 2> gpurun_out/bench_config3.err || exit 4
echo "== bench5"; timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_config5.json 2> gpurun_out/bench5.err || exit 5
echo "== dh7"; timeout -k 10 300 python bench.py --config dh7 --steps 5 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_dh7.json 2> gpurun_out/bench_dh7.err || exit 6
echo "== rocprof default bench"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- \
    python3 bench.py > gpurun_out/bench_under_rocprof.json 2> gpurun_out/bench_under_rocprof.err || exit 7
echo ROUND_DONE
echo "== PMC config 5"
PROF_NAME=c5 PROF_ARGS="--config 5 --swarms-per-gpu 2048 --iterations 100 --steps 1 --warmup 1 --cpu-seconds 0" bash tools/gpu_profile.sh || exit 8
echo PMC_DONE
if ls variants/c5_*.so >/dev/null 2>&1; then
  echo "== variants c5"
  timeout -k 10 400 python tools/variant_bench.py variants/c5_*.so --config 5 --swarms 2048 --iters 100 --rounds 3 \
      > gpurun_out/var_c5.txt 2>&1 || exit 9
fi
echo VARIANTS_DONE
