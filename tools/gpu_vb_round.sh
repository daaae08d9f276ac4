cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/variant_bench.py variants/libikpso_ub.so variants/libikpso_nsf.so --swarms 4096 --rounds 5 > gpurun_out/vb.log 2>&1; rc=$?; cat gpurun_out/vb.log | tail -4; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_round.sh
