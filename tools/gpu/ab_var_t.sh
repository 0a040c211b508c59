# correctness of each variant on the GEMM op tests, then the A/B of tools/gpu/ab_var.sh
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/abv
for v in "$@"; do
  VITMI_LIB=$PWD/transformer-stm_amd/build/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "linear or gemm" > gpurun_out/abv/tests_$v.log 2>&1
done
bash tools/gpu/ab_var.sh "$@"
