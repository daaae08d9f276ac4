#!/bin/bash
# Verification session: every GPU test, smoke, the default bench line, and the
# rocprofv3 kernel trace of the same default bench command (its average kernel
# duration must agree with the line's HIP-event kernel_ms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES="tests smoke bench" bash tools/gpu_check.sh || exit $?
echo "== rocprof default bench"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- \
    python3 bench.py > gpurun_out/bench_under_rocprof.log 2>&1 || exit 5
echo VERIFY_DONE
