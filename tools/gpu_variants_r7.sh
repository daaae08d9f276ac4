#!/bin/bash
# Config-3 experiment builds (variants/r7_*.so, tools/build_variants.sh REF7_ONLY) timed interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python tools/variant_bench.py variants/r7_*.so --config 3 --rounds 7 > gpurun_out/var_r7.txt 2>&1 || exit 3
echo VARIANTS_DONE
