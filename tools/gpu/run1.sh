set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -x -q > gpurun_out/ops.log 2>&1
timeout -k 10 120 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1
for v in v0 v1; do
  VITMI_LIB=$PWD/transformer-stm_amd/build/variants/$v.so timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/gb_$v.log 2>&1
done
timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/gb_v2.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_quick.log 2>&1
timeout -k 10 200 python tools/torch_prof.py 64 > gpurun_out/tprof.log 2>&1
