# Kernel + step A/B of library variants against the in-tree build (same box, alternating):
#   bash tools/gpu/kab.sh TAG "PYTEST_K" "TOOL CMD" VAR1 [VAR2 ...]
# runs the GPU tests selected by PYTEST_K, then TOOL CMD and a 10-step bench for each build, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=$1; k=$2; tool=$3; shift 3
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest tests -m gpu -k "$k" -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || exit 1
for round in 1 2; do
  for v in base "$@"; do
    lib=""; [ $v != base ] && lib=$PWD/transformer-stm_amd/variants/$v.so
    VITMI_LIB=$lib timeout -k 10 120 $tool > gpurun_out/$tag/tool_${v}_$round.log 2>&1 || exit 1
    VITMI_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 10 --warmup 3 > gpurun_out/$tag/step_${v}_$round.log 2>&1 || exit 1
  done
done
