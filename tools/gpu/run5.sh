set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
VITMI_GEMM_TAIL=0 timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/gb_v6_notail.log 2>&1
timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/gb_v6_tail.log 2>&1
VITMI_LIB=$PWD/transformer-stm_amd/build/variants/v1.so timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/gb_v1b.log 2>&1
