# bf16f8 knob with the qkv GEMM plain bf16 (the default) vs split: knob tests, then C3 bench
# lines of both, twice.   bash tools/gpu/qkv_knob.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out/$tag
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_model.py tests/test_gpu_f8.py -x -v -s -k "knob or f8" --timeout 240 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || { tail -30 gpurun_out/$tag/test.log; exit 1; }
grep -E "passed|failed|logits" gpurun_out/$tag/test.log | tail -20
for i in 1 2; do
  for q in no yes; do
    timeout -k 10 300 python3 bench.py --config c3 --dtype bf16f8 --split-qkv $q --steps 5 --warmup 2 --no-secondary \
        --no-evidence --no-cpu-baseline > gpurun_out/$tag/q$q$i.json 2>/dev/null || exit 1
    echo "split-qkv $q: $(grep -o '"value": [0-9.]*' gpurun_out/$tag/q$q$i.json)"
  done
done
