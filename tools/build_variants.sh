#!/bin/bash
# Experiment builds of libikpso.so for tools/variant_bench.py: one topology
# subset, one build directory and one output per variant.
#   tools/build_variants.sh SUBSET NAME [EXTRA FLAGS...]      (current tree)
#   HEAD_TREE=/path/to/checkout tools/build_variants.sh ...    (another tree)
# SUBSET: SERIAL20_ONLY | REF7_ONLY | REF7_SERIAL20 | DH_ONLY.  Output: vlib6/NAME.so (git-ignored).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SUBSET=$1; NAME=$2; shift 2
SRC=${HEAD_TREE:-$ROOT}/inverse-kinematics-pso-research_amd/csrc
mkdir -p "$ROOT/vlib6"
make -C "$SRC" -j8 BUILD="/tmp/ikpso_var_$NAME" OUT="$ROOT/vlib6/$NAME.so" \
     EXTRA="-DIKPSO_EXPERIMENT_$SUBSET $*" > "/tmp/ikpso_var_$NAME.log" 2>&1 || { tail -30 "/tmp/ikpso_var_$NAME.log"; exit 1; }
echo "built vlib6/$NAME.so"
