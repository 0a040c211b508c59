# Round-3 evidence: full GPU suite (skip reasons listed), then the default bench line (evidence
# legs + secondary C5/C2 lines) and a rocprofv3 kernel summary of the same step.
#   bash tools/gpu/run_r03.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-r03}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rs --timeout 180 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || exit 1
bash tools/gpu/bench.sh $tag
