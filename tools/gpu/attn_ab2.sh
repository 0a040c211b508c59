# Attention kernel A/B at the C3 and C5 shapes: tests (in-tree build), then tools/attn_bench.py for
# the in-tree build and a variant library, twice each, then both bench lines.
#   bash tools/gpu/attn_ab2.sh TAG VARIANT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=$1; var=$2
mkdir -p gpurun_out/$tag
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_cvt.py -x -q -k "attention or attn or vit_b or c1 or c5 or deterministic or knob or cvt" --timeout 240 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || { tail -30 gpurun_out/$tag/test.log; exit 1; }
tail -1 gpurun_out/$tag/test.log
for i in 1 2; do
  for shape in "256 197 12" "64 577 16"; do
    timeout -k 10 120 python3 tools/attn_bench.py $shape > gpurun_out/$tag/new$i.log 2>&1 || exit 1
    echo "new  $shape: $(grep -v amdgpu.ids gpurun_out/$tag/new$i.log | tr '\n' ' ')"
    VITMI_LIB=transformer-stm_amd/variants/$var.so timeout -k 10 120 python3 tools/attn_bench.py $shape > gpurun_out/$tag/base$i.log 2>&1 || exit 1
    echo "base $shape: $(grep -v amdgpu.ids gpurun_out/$tag/base$i.log | tr '\n' ' ')"
  done
done
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-evidence > gpurun_out/$tag/new_bench$i.json 2>/dev/null || exit 1
  VITMI_LIB=transformer-stm_amd/variants/$var.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-evidence > gpurun_out/$tag/base_bench$i.json 2>/dev/null || exit 1
  python3 - gpurun_out/$tag/new_bench$i.json gpurun_out/$tag/base_bench$i.json <<'PY'
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).readline())
    sec=d.get('secondary',{})
    print(f.split('/')[-1], 'c3', d['value'], ' '.join(f"{k} {v.get('value')}" for k,v in sec.items()))
PY
done
