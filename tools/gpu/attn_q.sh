set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/att
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/att/tests_q.log 2>&1
timeout -k 10 120 python tools/attn_bench.py > gpurun_out/att/ab_q.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/att/bench_q.log 2>&1
