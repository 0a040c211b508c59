# GPU test suite (one process, per-test thread timeout): bash tools/gpu/test.sh [pytest -k expr]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread $K > gpurun_out/test.log 2>&1
