#!/bin/bash
# Wave-priority levelling in the 4-wave kernels (full-library variants built with
# IKPSO_PRIO_LEVEL=2, 4 or 2 levels) against the shipped build: the folded DH arm
# through bench.py (IKPSO_LIB selects the library) and config 3 interleaved in
# one process (tools/variant_bench.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=inverse-kinematics-pso-research_amd/ikpso/_lib/libikpso.so
for v in "$LIB" variants/full_p2L4.so variants/full_p2L2.so "$LIB"; do
  n=$(basename "$v" .so)
  echo "== dh7 $n"
  IKPSO_LIB=$PWD/$v timeout -k 10 300 python bench.py --config dh7 --steps 5 --warmup 1 --cpu-seconds 0 \
      >> gpurun_out/var_dh7.jsonl 2>> gpurun_out/var_dh7.err || exit 2
done
echo "== config 3"
timeout -k 10 400 python tools/variant_bench.py "$LIB" variants/full_p2L4.so variants/full_p2L2.so --config 3 --rounds 5 \
    > gpurun_out/var_r7.txt 2>&1 || exit 3
echo VARIANTS_DONE
