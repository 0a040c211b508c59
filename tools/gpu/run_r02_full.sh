# Round-2 evidence: full GPU suite (skip reasons listed), then the default bench line with its
# evidence legs and a rocprofv3 kernel summary of the same step (tools/gpu/bench.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-r02_full}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rs --timeout 180 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || exit 1
bash tools/gpu/bench.sh $tag
