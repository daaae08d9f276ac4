cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
ARGS="--swarms-per-gpu 2048 --steps 1 --warmup 1 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU -d gpurun_out/prof_x1 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_x1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 -d gpurun_out/prof_x2 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_x2.log 2>&1
echo rc=$?
