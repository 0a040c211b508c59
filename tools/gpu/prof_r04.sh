# rocprofv3 kernel summary of a short bench run + the torch.profiler host call sites of the
# non-vitmi kernels.   bash tools/gpu/prof_r04.sh TAG [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-prof}; shift
mkdir -p gpurun_out/$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/$tag/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 5 --warmup 2 "$@" > gpurun_out/$tag/prof.log 2>&1 && \
python3 tools/prof_summary.py "$(find gpurun_out/$tag/prof -name 'run_kernel_stats.csv' | head -1)" 7 > gpurun_out/$tag/summary.txt && \
timeout -k 10 200 python3 tools/torch_prof.py 256 > gpurun_out/$tag/torch_prof.txt 2>&1
rc=$?
head -45 gpurun_out/$tag/summary.txt
exit $rc
