# streamed attention (N > 256) change: op parity (both paths), C5 model parity, kernel timing, C5 bench
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/ac5
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k attention -x -q --timeout 120 --timeout-method thread > gpurun_out/ac5/ops.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k c5 -x -q --timeout 200 --timeout-method thread > gpurun_out/ac5/model.log 2>&1
timeout -k 10 120 python tools/attn_bench.py 64 577 16 > gpurun_out/ac5/attn.log 2>&1
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/ac5/bench.log 2>&1
