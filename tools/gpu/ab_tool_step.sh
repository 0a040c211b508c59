# alternating rounds of one tool and the 10-step bench for the in-tree build and each variant:
#   bash tools/gpu/ab_tool_step.sh TAG "TOOL CMD" VAR1 [VAR2 ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=$1; tool=$2; shift 2
mkdir -p gpurun_out/$tag
for round in 1 2; do
  for v in base "$@"; do
    lib=""; [ $v != base ] && lib=$PWD/transformer-stm_amd/variants/$v.so
    VITMI_LIB=$lib timeout -k 10 120 $tool > gpurun_out/$tag/tool_${v}_$round.log 2>&1 || exit 1
    VITMI_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 10 --warmup 3 > gpurun_out/$tag/step_${v}_$round.log 2>&1 || exit 1
  done
done
