# Per-kernel A/B inside the bench step: a rocprofv3 kernel summary of the step for the in-tree
# build and each variants/NAME.so (two alternating rounds), plus the GPU tests selected by -k:
#   bash tools/gpu/prof_ab.sh TAG "PYTEST_K" VAR1 [VAR2 ...]   -> gpurun_out/TAG/sum_<build>_<round>.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=$1; k=$2; shift 2
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest tests -m gpu -k "$k" -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || exit 1
for round in 1 2; do
  for v in base "$@"; do
    lib=""; [ $v != base ] && lib=$R/transformer-stm_amd/variants/$v.so
    d=$R/gpurun_out/$tag/prof_${v}_$round
    VITMI_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-evidence --steps 5 --warmup 2 > gpurun_out/$tag/bench_${v}_$round.log 2>&1 || exit 1
    python3 tools/prof_summary.py "$(find $d -name 'run_kernel_stats.csv' | head -1)" 7 > gpurun_out/$tag/sum_${v}_$round.txt || exit 1
  done
done
