# round-1 measurement pass: full bench line (with cpu_baseline), rocprof kernel stats of the
# same command, and the two PMC passes for the dominant GEMM's HBM traffic.
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 600 python bench.py > gpurun_out/r3/bench.json 2> gpurun_out/r3/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r3/prof.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/r3/pmc_fetch -o run --output-format csv -- python3 tools/gemm_one.py fc1_gelu 5 > gpurun_out/r3/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/r3/pmc_write -o run --output-format csv -- python3 tools/gemm_one.py fc1_gelu 5 > gpurun_out/r3/pmc_write.log 2>&1
