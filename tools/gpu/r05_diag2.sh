set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r05_diag2
timeout -k 10 400 python3 tools/diag_grad_precision.py > gpurun_out/r05_diag2/grad.log 2>&1 || { tail -20 gpurun_out/r05_diag2/grad.log; exit 1; }
