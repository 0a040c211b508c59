# rocprofv3 kernel tables of the bench step under each environment setting:
#   bash tools/gpu/env_prof.sh TAG "VAR=VAL ..." ["VAR=VAL ..." ...] -> gpurun_out/TAG/sum_<i>.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=$1; shift
mkdir -p gpurun_out/$tag
i=0
for e in "$@"; do
  i=$((i+1))
  d=$R/gpurun_out/$tag/prof_$i
  export $e
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 5 --warmup 2 > gpurun_out/$tag/bench_$i.log 2>&1 || exit 1
  python3 tools/prof_summary.py "$(find $d -name 'run_kernel_stats.csv' | head -1)" 7 > gpurun_out/$tag/sum_$i.txt || exit 1
done
