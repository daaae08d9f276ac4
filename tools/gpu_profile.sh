#!/bin/bash
# rocprofv3 kernel trace + PMC passes (one counter group per pass; no tracing
# domains combined with --pmc) for a bench workload.  Outputs in
# gpurun_out/<PROF_NAME>_{trace,valu,fetch,write,cycles}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${PROF_ARGS:-"--swarms-per-gpu 2048 --steps 2 --warmup 1 --cpu-seconds 0"}
NAME=${PROF_NAME:-prof}
run() {  # run PASS ROCPROF_ARGS...
  local pass=$1; shift
  echo "== $NAME $pass"
  timeout -k 10 600 rocprofv3 "$@" -d "gpurun_out/${NAME}_$pass" -o run --output-format csv -- python3 bench.py $ARGS \
    > "gpurun_out/${NAME}_$pass.log" 2>&1
  local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/${NAME}_$pass.log"; exit $rc; }
}
# the library build the counters are measured on (bench.py marks a roofline whose counters came from
# another build as stale)
python3 -c "import sys; sys.path.insert(0, 'inverse-kinematics-pso-research_amd'); import ikpso; print(ikpso.build_id())" \
  > "gpurun_out/${NAME}_build_id.txt" || exit 9
run trace --kernel-trace --stats
run valu --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run cycles --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY
# issue stalls on the LDS and the scalar/LDS instruction mix (round 6)
run waits --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES
echo ALL_DONE
