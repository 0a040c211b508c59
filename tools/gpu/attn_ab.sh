# Attention A/B: GPU attention/model tests, then the kernels timed in isolation for the in-tree
# build against a variant library (VITMI_LIB), then the default bench line.
#   bash tools/gpu/attn_ab.sh TAG VARIANT_NAME "VARIANT_ENV"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-attn_ab}; var=$2; venv=$3
mkdir -p gpurun_out/$tag
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -k "attention or attn or vit_b or c1 or c2 or c5 or deterministic or knob" --timeout 240 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || { tail -30 gpurun_out/$tag/test.log; exit 1; }
tail -2 gpurun_out/$tag/test.log
for i in 1 2; do
  timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/$tag/new$i.log 2>&1 || exit 1
  env VITMI_LIB=transformer-stm_amd/variants/$var.so $venv timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/$tag/base$i.log 2>&1 || exit 1
done
head -50 gpurun_out/$tag/new*.log gpurun_out/$tag/base*.log
bash tools/gpu/bench.sh $tag --no-secondary
cut -c1-400 gpurun_out/$tag/bench.json
grep -E "attn|total" gpurun_out/$tag/summary.txt
