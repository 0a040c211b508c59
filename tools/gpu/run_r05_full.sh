# Round-5 evidence: the whole -m gpu suite (skip reasons listed), then the default bench line
# (evidence legs + secondary lines) and a rocprofv3 kernel summary of the same step.
#   bash tools/gpu/run_r05_full.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-r05}
mkdir -p gpurun_out/$tag
timeout -k 10 120 python3 tools/host_overhead.py > gpurun_out/$tag/host.log 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rs --timeout 240 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || { tail -30 gpurun_out/$tag/test.log; exit 1; }
tail -3 gpurun_out/$tag/test.log
bash tools/gpu/bench.sh $tag
rc=$?
cut -c1-600 gpurun_out/$tag/bench.json
exit $rc
