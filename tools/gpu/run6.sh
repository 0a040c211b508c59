set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q > gpurun_out/tests7.log 2>&1
VITMI_GEMM_TAIL=0 timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/gb_v7_notail.log 2>&1
timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/gb_v7_tail.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_quick7.log 2>&1
VITMI_GEMM_TAIL=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_quick7_notail.log 2>&1
mkdir -p gpurun_out/r7
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/r7/pmc_write -o run --output-format csv -- python3 tools/gemm_one.py fc1_gelu 5 > gpurun_out/r7/pmc_write.log 2>&1
