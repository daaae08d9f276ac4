#!/bin/bash
# build_variants.sh NAME "FLAGS" [NAME "FLAGS" ...] -> variants/libikpso_NAME.so
cd "$(dirname "$0")/../inverse-kinematics-pso-research_amd/csrc"
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s -j8 OUT=../../variants/libikpso_$name.so BUILD=_build_$name EXTRA="$flags" >/tmp/bv_$name.log 2>&1 &
  pids+=($!)
done
rc=0; for p in "${pids[@]}"; do wait $p || rc=1; done; exit $rc
