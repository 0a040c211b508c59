# bf16f8 and bf16x3 steps: bench lines and rocprofv3 kernel summaries (round 6)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=${1:-r06_f8prof}
mkdir -p gpurun_out/$tag
for d in bf16f8 bf16x3; do
  timeout -k 10 200 python3 bench.py --dtype $d --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
      > gpurun_out/$tag/bench_$d.json 2> gpurun_out/$tag/bench_$d.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/prof_$d -o run --output-format csv -- \
      python3 bench.py --dtype $d --no-cpu-baseline --no-evidence --no-secondary --no-parity --steps 3 --warmup 2 \
      > gpurun_out/$tag/prof_$d.log 2>&1 || exit 1
  python3 tools/prof_summary.py "$(find gpurun_out/$tag/prof_$d -name 'run_kernel_stats.csv' | head -1)" 5 \
      > gpurun_out/$tag/summary_$d.txt || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_$d.json'));print('$d', d['value'], d['ms_per_step'], d['phases_ms'], d['parity']['logits_max_abs'])"
  head -22 gpurun_out/$tag/summary_$d.txt
done
