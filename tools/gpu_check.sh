#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a crash/timeout (not a plain test
# failure) ends the script so nothing else touches the GPU after a fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "   rc=$rc"; tail -5 "gpurun_out/$name.log"
  return $rc
}
STAGES=${STAGES:-tests smoke bench prof}
for s in $STAGES; do
  case $s in
    tests) step gpu_tests 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider; ok $? || exit 2 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 3 ;;
    bench) step bench 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 || exit 4 ;;
    prof)  cd /tmp && step_dir="$GRAFT_REPO_ROOT" && cd "$step_dir" &&
           step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
                python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 || exit 5 ;;
  esac
done
echo ALL_DONE
