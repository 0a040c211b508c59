# forward attention: Q rows through the V image by LDS-DMA (VITMI_ATTN_FWD_QLDS=1) vs per-lane row
# loads; attention tests on the variant, attn_bench and the C3 step, 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_qlds}
mkdir -p gpurun_out/$tag
VITMI_LIB=$V/aqlds.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_f8.py -m gpu -x -q \
    --timeout 180 --timeout-method thread -k "attention or attn" > gpurun_out/$tag/test.log 2>&1 || { tail -30 gpurun_out/$tag/test.log; exit 1; }
tail -1 gpurun_out/$tag/test.log
for r in 1 2; do
  for v in base aqlds; do
    L=""; [ $v != base ] && L=$V/$v.so
    echo "== $v $r"; VITMI_LIB=$L timeout -k 10 120 python3 tools/attn_bench.py 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "step $v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['forward'])")"
  done
done
