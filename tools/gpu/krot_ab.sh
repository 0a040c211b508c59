# Weight-gradient K-rotation A/B: the default bench step (no evidence legs) and its rocprofv3
# kernel summary for the in-tree build with VITMI_WGRAD_KROT settings, against a base variant.
#   bash tools/gpu/krot_ab.sh TAG "R,S" ["R,S" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=$1; shift
mkdir -p gpurun_out/$tag
VITMI_WGRAD_KROT=4,2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -x -q -k "wgrad or gemm or linear" --timeout 120 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || { tail -20 gpurun_out/$tag/test.log; exit 1; }
tail -1 gpurun_out/$tag/test.log
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/$name -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 10 --warmup 3 > gpurun_out/$tag/$name.json 2> gpurun_out/$tag/$name.err || return 1
  python3 tools/prof_summary.py "$(find gpurun_out/$tag/$name -name 'run_kernel_stats.csv' | head -1)" 13 > gpurun_out/$tag/$name.sum
  printf '%-10s %s\n' $name "$(cut -c1-120 gpurun_out/$tag/$name.json | grep -o '"value": [0-9.]*')"
  grep -E "gemm256_kernel<false, false, 100|splitk|total" gpurun_out/$tag/$name.sum
}
for rep in 1 2; do
  run base$rep VITMI_LIB=transformer-stm_amd/variants/base.so || exit 1
  run off$rep VITMI_WGRAD_KROT=0 || exit 1
  for k in "$@"; do run k${k/,/_}_$rep VITMI_WGRAD_KROT=$k || exit 1; done
done
