# Bench line (+ evidence legs) and a rocprofv3 kernel summary of the same step:
#   bash tools/gpu/bench.sh TAG [bench args...]   -> gpurun_out/TAG/{bench.json,summary.txt,...}
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=${1:-cur}; shift
mkdir -p gpurun_out/$tag
timeout -k 10 600 python3 bench.py "$@" > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 5 --warmup 2 "$@" > gpurun_out/$tag/prof.log 2>&1 && \
python3 tools/prof_summary.py "$(find gpurun_out/$tag/prof -name 'run_kernel_stats.csv' | head -1)" 7 \
    > gpurun_out/$tag/summary.txt
