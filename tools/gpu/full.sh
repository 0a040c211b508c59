# full GPU test suite, GEMM microbench, quick bench
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/full
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full/tests.log 2>&1
timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/full/gb.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/full/bench.log 2>&1
