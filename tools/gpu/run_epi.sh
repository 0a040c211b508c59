set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/epi_test.log 2>&1 || exit 1
VITMI_LIB=$PWD/transformer-stm_amd/variants/stamps_lds.so timeout -k 10 200 python3 tools/gemm_stamps.py > gpurun_out/stamps_lds.log 2>&1 || exit 1
bash tools/gpu/ab.sh ab_epi "python3 bench.py --no-cpu-baseline --no-evidence --steps 10 --warmup 3" gemm_old
