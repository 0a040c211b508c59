set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/att
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/att/tests.log 2>&1
VITMI_ATTN_PP=0 timeout -k 10 120 python tools/attn_bench.py > gpurun_out/att/ab0.log 2>&1
VITMI_ATTN_PP=1 timeout -k 10 120 python tools/attn_bench.py > gpurun_out/att/ab1.log 2>&1
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/att/tests_all.log 2>&1
VITMI_ATTN_PP=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/att/bench0.log 2>&1
VITMI_ATTN_PP=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/att/bench1.log 2>&1
