set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/dgb
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_cvt_model.py -x -v --timeout 120 --timeout-method thread -k "fused_bias or model or cvt or mlp or block" > gpurun_out/dgb/tests.log 2>&1
GEMM_BENCH_ONLY=dGELU timeout -k 10 120 python tools/gemm_bench.py 20 > gpurun_out/dgb/gemm.txt 2>&1
for i in 1 2; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/dgb/bench.txt 2>&1; done
