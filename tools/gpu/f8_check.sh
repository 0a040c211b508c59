# bf16f8 knob check: its op tests, the model knob tests, the C3 bf16f8 bench line and the GEMM
# stamps (VITMI_LIB=variants/stamps.so).   bash tools/gpu/f8_check.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-f8check}
mkdir -p gpurun_out/$tag
timeout -k 10 200 python3 -m pytest tests/test_gpu_f8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/ops.log 2>&1 || { tail -30 gpurun_out/$tag/ops.log; exit 1; }
tail -1 gpurun_out/$tag/ops.log
timeout -k 10 400 python3 -m pytest tests/test_gpu_model.py -x -q -s -k "bf16f8" --timeout 300 --timeout-method thread > gpurun_out/$tag/model.log 2>&1 || { tail -30 gpurun_out/$tag/model.log; exit 1; }
grep -E "logits|passed|failed" gpurun_out/$tag/model.log
timeout -k 10 300 python3 bench.py --config c3 --dtype bf16f8 --steps 5 --warmup 2 --no-secondary --no-evidence \
    --no-cpu-baseline > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || exit 1
cut -c1-200 gpurun_out/$tag/bench.json
if [ -f transformer-stm_amd/variants/stamps.so ]; then
  VITMI_LIB=transformer-stm_amd/variants/stamps.so timeout -k 10 200 python3 tools/gemm_stamps.py > gpurun_out/$tag/stamps.log 2>&1 || exit 1
  grep -v "per-" gpurun_out/$tag/stamps.log | head -5
fi
