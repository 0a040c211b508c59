set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q > gpurun_out/tests8.log 2>&1
timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/gb_v8.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_quick8.log 2>&1
