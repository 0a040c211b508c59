# The bf16f8 knob against bf16x3: bench lines (C3, 5 timed steps) and a kernel summary of each.
#   bash tools/gpu/f8_bench.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=${1:-f8bench}
mkdir -p gpurun_out/$tag
for d in bf16f8 bf16x3; do
  timeout -k 10 300 python3 bench.py --config c3 --dtype $d --steps 5 --warmup 2 --no-secondary --no-evidence \
      --no-cpu-baseline > gpurun_out/$tag/bench_$d.json 2> gpurun_out/$tag/bench_$d.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/prof_$d -o run --output-format csv -- \
      python3 bench.py --config c3 --dtype $d --no-cpu-baseline --no-evidence --no-secondary --steps 3 --warmup 2 \
      > gpurun_out/$tag/prof_$d.log 2>&1 || exit 1
  python3 tools/prof_summary.py "$(find gpurun_out/$tag/prof_$d -name 'run_kernel_stats.csv' | head -1)" 5 \
      > gpurun_out/$tag/summary_$d.txt || exit 1
  cut -c1-200 gpurun_out/$tag/bench_$d.json
  head -14 gpurun_out/$tag/summary_$d.txt
done
