# Adam per gradient bucket on a side stream beside the backward (--adam-overlap 1) vs one launch
# after it: optimizer / dp tests, then the C3 step, 3 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=${1:-r06_aov}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_optim.py tests/test_gpu_dp.py \
    > gpurun_out/$tag/tests.txt 2>&1 || { tail -30 gpurun_out/$tag/tests.txt; exit 1; }
tail -1 gpurun_out/$tag/tests.txt
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity --adam-overlap $v > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "ov=$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms'])")"
  done
done
