cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1; grep -i "icache\|SQC_" gpurun_out/pmc_list.txt | head -20
L=inverse-kinematics-pso-research_amd/ikpso/_lib/libikpso.so
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d gpurun_out/icache5 -o run --output-format csv -- python3 tools/variant_bench.py $L --config 5 --swarms 512 --iters 50 --rounds 1 > gpurun_out/icache5.log 2>&1; echo rc5=$?
