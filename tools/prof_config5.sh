#!/bin/bash
# rocprofv3 kernel trace + HBM counters of the streaming kernels on BASELINE
# config 5 (20-joint chain, 4096 particles), shortened to 50 iterations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${PROF_ARGS:-"--config 5 --steps 1 --warmup 1 --iterations 50 --swarms-per-gpu 2048 --cpu-seconds 0"}
echo "== bench"; timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/c5_bench.log 2>&1 || exit 3
tail -1 gpurun_out/c5_bench.log | cut -c1-300
run() {  # run NAME ROCPROF_ARGS...
  local name=$1; shift
  echo "== $name"
  timeout -k 10 300 rocprofv3 "$@" -d "gpurun_out/c5_$name" -o run --output-format csv -- python3 bench.py $ARGS \
    > "gpurun_out/c5_$name.log" 2>&1
  local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/c5_$name.log"; exit $rc; }
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run valu --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
echo ALL_DONE
