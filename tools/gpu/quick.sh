# GEMM op tests + GEMM microbench + quick bench of the in-tree library
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "linear or gemm" > gpurun_out/q/tests_ops.log 2>&1
timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/q/gb.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/q/bench.log 2>&1
