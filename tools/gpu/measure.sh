# round measurement pass: full bench line (with cpu_baseline), rocprofv3 kernel stats of the
# same workload, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) of the dominant fc1 GEMM.
# usage: bash tools/gpu/measure.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=${1:-m}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/$tag/prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/$tag/pmc_fetch -o run --output-format csv -- python3 tools/gemm_one.py fc1_gelu 5 > gpurun_out/$tag/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/$tag/pmc_write -o run --output-format csv -- python3 tools/gemm_one.py fc1_gelu 5 > gpurun_out/$tag/pmc_write.log 2>&1
