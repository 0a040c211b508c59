# GPU tests of the GEMM/attention/model path, then per-kernel timings (attention, every ViT GEMM
# shape) and the step A/B, each for the in-tree build and the variants named:
#   bash tools/gpu/run_full_ab.sh TAG VAR1 [VAR2 ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || exit 1
for v in base "$@"; do
  lib=""; [ $v != base ] && lib=$PWD/transformer-stm_amd/variants/$v.so
  VITMI_LIB=$lib timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/$tag/attn_$v.log 2>&1 || exit 1
  VITMI_LIB=$lib timeout -k 10 180 python3 tools/gemm_shapes.py > gpurun_out/$tag/gemm_$v.log 2>&1 || exit 1
done
bash tools/gpu/ab.sh $tag "python3 bench.py --no-cpu-baseline --no-evidence --steps 10 --warmup 3" "$@"
