# attention parity tests, then kernel timing and the step A/B against the variants named
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/$tag/attn_base.log 2>&1 || exit 1
for v in "$@"; do
  VITMI_LIB=$PWD/transformer-stm_amd/variants/$v.so timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/$tag/attn_$v.log 2>&1 || exit 1
done
bash tools/gpu/ab.sh $tag "python3 bench.py --no-cpu-baseline --no-evidence --steps 10 --warmup 3" "$@"
