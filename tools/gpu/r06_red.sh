# split-K reductions with the slab loads issued together (in-tree) vs one load-then-add at a time
# (redold): wgrad tests, then the C3 step and the reduce kernels' times (rocprofv3), 3 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_red}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "wgrad or split or linear" tests \
    > gpurun_out/$tag/tests.txt 2>&1 || { tail -30 gpurun_out/$tag/tests.txt; exit 1; }
tail -1 gpurun_out/$tag/tests.txt
for r in 1 2 3; do
  for v in base redold; do
    L=""; [ $v != base ] && L=$V/$v.so
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['backward'])")"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in base redold; do
  L=""; [ $v != base ] && L=$V/$v.so
  VITMI_LIB=$L VITMI_WGRAD_STREAM=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$tag/prof_$v -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-secondary --no-evidence --no-cpu-baseline --no-parity > /dev/null 2>&1 || exit 1
  f=$(find $GRAFT_REPO_ROOT/gpurun_out/$tag/prof_$v -name "*kernel_stats.csv" | head -1)
  echo "$v: $(grep -E 'splitk_reduce' $f | cut -d, -f1-5 | tr '\n' ' ')"
done
