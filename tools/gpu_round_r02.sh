#!/bin/bash
# Round-2 GPU session: every GPU test, smoke, the default bench line, the DH
# bench lines (folded / Euler with mask / locked axes), config 5, then the
# rocprofv3 kernel traces + PMC passes bench.py's roofline reads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="tests smoke bench" bash tools/gpu_check.sh || exit $?
for c in dh7 dh7-nofold dh7-locked; do
  echo "== bench $c"
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --cpu-seconds 6 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 6
done
echo "== bench5"; timeout -k 10 600 python bench.py --config 5 --steps 2 --warmup 1 --cpu-seconds 6 > gpurun_out/bench5.json 2> gpurun_out/bench5.err || exit 7
bash tools/gpu_profile_set.sh > gpurun_out/profset.log 2>&1 || exit 8
echo ROUND_DONE
