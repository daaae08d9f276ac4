cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_mask.py tests/test_gpu_dh.py -p no:cacheprovider > gpurun_out/mask_tests.log 2>&1
for c in dh7 dh7-nofold dh7-locked; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 4 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 3
done
