# attention pipelining experiment: attention tests on the in-tree build (the variant), then
# tools/attn_bench.py in-tree vs variants/base.so, twice.   bash tools/gpu/swp_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out/$tag
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -k "attention or attn or vit_b_bf16 or c1_ or knob" --timeout 240 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || { tail -30 gpurun_out/$tag/test.log; exit 1; }
tail -1 gpurun_out/$tag/test.log
for i in 1 2; do
  echo "new : $(timeout -k 10 100 python3 tools/attn_bench.py 2>&1 | grep seq)" || exit 1
  echo "base: $(VITMI_LIB=transformer-stm_amd/variants/base.so timeout -k 10 100 python3 tools/attn_bench.py 2>&1 | grep seq)" || exit 1
done
