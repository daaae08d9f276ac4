#!/bin/bash
# Interleaved variant timing on the GPU box: tools/gpu_var.sh OUTNAME CONFIG SWARMS ITERS LIB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=$1; cfg=$2; sw=$3; it=$4; shift 4
echo "== variants $out"
IKPSO_ALLOW_STALE=1 timeout -k 10 600 python -u tools/variant_bench.py "$@" --config "$cfg" --swarms "$sw" --iters "$it" \
  --rounds 5 > "gpurun_out/var_$out.txt" 2>&1; rc=$?; cat "gpurun_out/var_$out.txt"; exit $rc
