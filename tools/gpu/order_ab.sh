# Backward GEMM-order A/B (VITMI_MLP_BWD_ORDER): bench step + rocprofv3 kernel summary per order.
#   bash tools/gpu/order_ab.sh TAG a b c
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=$1; shift
mkdir -p gpurun_out/$tag
for rep in 1 2; do
  for o in "$@"; do
    name=$o$rep
    VITMI_MLP_BWD_ORDER=$o timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/$name -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 10 --warmup 3 > gpurun_out/$tag/$name.json 2> gpurun_out/$tag/$name.err || exit 1
    python3 tools/prof_summary.py "$(find gpurun_out/$tag/$name -name 'run_kernel_stats.csv' | head -1)" 13 > gpurun_out/$tag/$name.sum
    printf '%-6s %s\n' $name "$(cut -c1-120 gpurun_out/$tag/$name.json | grep -o '"value": [0-9.]*')"
    grep -E "gemm256|total" gpurun_out/$tag/$name.sum | head -8
  done
done
