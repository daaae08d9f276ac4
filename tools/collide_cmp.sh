#!/bin/bash
# Collider-term kernel time at full size (bench.py --colliders {init03,far4}, 4096 x 1024 x 500) for the
# product library and vlib6/ variants, one box: VARIANTS="product coll_vN ..." bash tools/collide_cmp.sh
mkdir -p gpurun_out
for v in ${VARIANTS:-product coll_v1 coll_v3}; do
  for c in init03 far4 far4keep; do
    if [ $v = product ]; then L=""; else L="IKPSO_LIB=vlib6/$v.so IKPSO_ALLOW_STALE=1"; fi
    K=""; [ $c = far4keep ] && K="IKPSO_KEEP_FAR_COLLIDERS=1"; c=${c%keep}
    env $L $K timeout -k 10 300 python bench.py --colliders $c --steps 2 --warmup 1 --extra-steps 0 --frames 0 --reference-steps 0 --cpu-seconds 0 > gpurun_out/cmp_${v}_$c${K:+_keep}.log 2>&1 || exit 3
    echo "$v $c $K $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/cmp_${v}_$c${K:+_keep}.log | head -1)"
  done
done
