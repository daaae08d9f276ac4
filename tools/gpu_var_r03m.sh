#!/bin/bash
# Round 3: full-record polls in the cooperative exchange (variants lat_* = config 2, c5_* = config 5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export IKPSO_ALLOW_STALE=1
timeout -k 10 300 python -u tools/variant_bench.py variants/lat_*.so --config 3 --swarms 1 --rounds 7 > gpurun_out/var_lat_pf.txt 2>&1 || exit 2
timeout -k 10 400 python -u tools/variant_bench.py variants/c5_*.so --config 5 --swarms 2048 --iters 100 --rounds 5 > gpurun_out/var_c5_pf.txt 2>&1 || exit 3
grep -v amdgpu gpurun_out/var_lat_pf.txt gpurun_out/var_c5_pf.txt
