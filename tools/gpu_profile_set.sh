#!/bin/bash
# Kernel trace + PMC passes (tools/gpu_profile.sh) for the bench workloads whose
# per-update counters bench.py's roofline reads: config 3, the folded DH arm and
# config 5.  Each workload's passes stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PROF_NAME=c3 PROF_ARGS="--swarms-per-gpu 2048 --steps 2 --warmup 1 --cpu-seconds 0" bash tools/gpu_profile.sh || exit 1
PROF_NAME=dh7 PROF_ARGS="--config dh7 --swarms-per-gpu 2048 --steps 2 --warmup 1 --cpu-seconds 0" bash tools/gpu_profile.sh || exit 2
PROF_NAME=c5 PROF_ARGS="--config 5 --swarms-per-gpu 2048 --iterations 100 --steps 1 --warmup 1 --cpu-seconds 0" bash tools/gpu_profile.sh || exit 3
echo PROFILES_DONE
