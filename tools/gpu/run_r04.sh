# Round-4 check: the GPU suite (up to 5 failures reported), then a short bench line without the
# evidence legs.   bash tools/gpu/run_r04.sh TAG [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-r04}; shift
mkdir -p gpurun_out/$tag
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -rs --maxfail=5 --timeout 180 --timeout-method thread \
    > gpurun_out/$tag/test.log 2>&1
rc=$?
tail -5 gpurun_out/$tag/test.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 20 --warmup 5 "$@" \
    > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
cat gpurun_out/$tag/bench.json
exit $rc
