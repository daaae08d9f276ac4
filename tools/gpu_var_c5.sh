#!/bin/bash
# Config-5 experiment builds (variants/c5_*.so, tools/build_variants.sh SERIAL20_ONLY) timed interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export IKPSO_ALLOW_STALE=1
timeout -k 10 400 python -u tools/variant_bench.py variants/c5_*.so --config 5 --swarms 2048 --iters 100 --rounds 5 \
  > gpurun_out/var_c5.txt 2>&1; rc=$?; cat gpurun_out/var_c5.txt; exit $rc
