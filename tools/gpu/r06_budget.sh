# per-kernel step budget of the final tree with the weight gradients serial (VITMI_WGRAD_STREAM=0,
# so no launch shares the GPU with another): rocprofv3 kernel stats over 5 timed steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=${1:-r06_budget}
mkdir -p gpurun_out/$tag
VITMI_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --no-parity --steps 5 --warmup 2 > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/prof.log && \
python3 tools/prof_summary.py "$(find gpurun_out/$tag/prof -name 'run_kernel_stats.csv' | head -1)" 7 > gpurun_out/$tag/summary.txt && \
head -30 gpurun_out/$tag/summary.txt && cat gpurun_out/$tag/bench.json
