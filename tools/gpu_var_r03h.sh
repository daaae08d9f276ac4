#!/bin/bash
# Round 3: FAST draws as shifted bits (no v_cvt_f32_u32) vs the conversion, interleaved on the bench workloads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export IKPSO_ALLOW_STALE=1
timeout -k 10 300 python -u tools/variant_bench.py variants/r7_*.so --config 3 --rounds 5 > gpurun_out/var_r7_shift.txt 2>&1 || exit 2
timeout -k 10 300 python -u tools/variant_bench.py variants/c5_*.so --config 5 --swarms 2048 --iters 100 --rounds 5 > gpurun_out/var_c5_shift.txt 2>&1 || exit 3
timeout -k 10 300 python -u tools/variant_bench.py variants/dh_*.so --config dh7 --rounds 5 > gpurun_out/var_dh7_shift.txt 2>&1 || exit 4
cat gpurun_out/var_*_shift.txt
