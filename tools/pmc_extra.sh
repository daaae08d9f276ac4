#!/bin/bash
# Stall breakdown of the default bench kernel: two extra PMC passes (8 SQ
# counters each), each its own run.  Output: gpurun_out/prof_x{1,2}/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
ARGS="--swarms-per-gpu 2048 --steps 1 --warmup 1 --cpu-seconds 0 ${PMC_ARGS:-}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/prof_x1 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_x1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAVES SQ_BUSY_CU_CYCLES -d gpurun_out/prof_x2 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_x2.log 2>&1
echo rc=$?
