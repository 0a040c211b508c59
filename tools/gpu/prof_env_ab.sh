# rocprofv3 kernel tables of a short bench run under two values of an environment switch:
#   bash tools/gpu/prof_env_ab.sh TAG VAR VALUE_A VALUE_B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=$1; var=$2; shift 2
mkdir -p gpurun_out/$tag
for v in "$@"; do
  export $var=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/$tag/p_$v -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 5 --warmup 2 > gpurun_out/$tag/p_$v.log 2>&1 || exit 1
  python3 tools/prof_summary.py "$(find gpurun_out/$tag/p_$v -name 'run_kernel_stats.csv' | head -1)" 7 > gpurun_out/$tag/sum_$v.txt || exit 1
done
