# GPU tests (all), then alternating rounds of the isolated GEMM shapes, the attention kernels and
# the 10-step bench for the in-tree build and each variants/NAME.so:
#   bash tools/gpu/ab3.sh TAG VAR1 [VAR2 ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || exit 1
for round in 1 2; do
  for v in base "$@"; do
    lib=""; [ $v != base ] && lib=$PWD/transformer-stm_amd/variants/$v.so
    VITMI_LIB=$lib timeout -k 10 120 python3 tools/gemm_shapes.py > gpurun_out/$tag/gemm_${v}_$round.log 2>&1 || exit 1
    VITMI_LIB=$lib timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/$tag/attn_${v}_$round.log 2>&1 || exit 1
    VITMI_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 10 --warmup 3 > gpurun_out/$tag/step_${v}_$round.log 2>&1 || exit 1
  done
done
