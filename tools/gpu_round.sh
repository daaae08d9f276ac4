#!/bin/bash
# tests + bench (config 3) + config 5 + visualiser frame latency, each under its own limit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="tests bench" bash tools/gpu_check.sh || exit $?
echo "== bench5"; timeout -k 10 600 python bench.py --config 5 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/bench5.log 2>&1 || { tail -5 gpurun_out/bench5.log; exit 6; }
tail -1 gpurun_out/bench5.log | cut -c1-400
echo "== frame"; timeout -k 10 300 python tools/frame_bench.py > gpurun_out/frame.log 2>&1 || exit 7
cat gpurun_out/frame.log | grep calc
echo "== batch_c"; timeout -k 10 120 examples/_build/batch_c 4096 500 > gpurun_out/batch_c.log 2>&1 || exit 8
cat gpurun_out/batch_c.log
echo ROUND_DONE
