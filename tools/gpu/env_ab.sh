# GPU tests (all), then alternating rounds of the 10-step bench under each environment setting:
#   bash tools/gpu/env_ab.sh TAG "VAR=VAL ..." ["VAR=VAL ..." ...]   (first setting = "base")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || exit 1
for round in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 10 --warmup 3 > gpurun_out/$tag/step_${i}_$round.log 2>&1 || exit 1
  done
done
