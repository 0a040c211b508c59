# A/B timing of library variants (transformer-stm_amd/variants/NAME.so, tools/build_variant.sh)
# against the in-tree build, alternating runs:   bash tools/gpu/ab.sh TAG "CMD ARGS" VAR1 [VAR2 ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=$1; cmd=$2; shift 2
mkdir -p gpurun_out/$tag
for round in 1 2; do
  timeout -k 10 300 $cmd > gpurun_out/$tag/base_$round.log 2>&1 || exit 1
  for v in "$@"; do
    VITMI_LIB=$PWD/transformer-stm_amd/variants/$v.so timeout -k 10 300 $cmd > gpurun_out/$tag/${v}_$round.log 2>&1 || exit 1
  done
done
