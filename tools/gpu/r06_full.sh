# Round 6 full check: the whole -m gpu suite (one process, per-test thread timeouts), smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-r06_full}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread -rs \
    > gpurun_out/$tag/test.log 2>&1 || { tail -60 gpurun_out/$tag/test.log; exit 1; }
tail -4 gpurun_out/$tag/test.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 || { tail -20 gpurun_out/$tag/smoke.log; exit 1; }
tail -2 gpurun_out/$tag/smoke.log
