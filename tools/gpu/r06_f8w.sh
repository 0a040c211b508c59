# the bf16f8 knob's qkv GEMM with the weight-side correction alone (VITMI_BF16F8W): kernel tests, the
# ViT-B depth-12 parity test in every qkv form, smoke, and the C3 bf16f8 step per qkv form
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=${1:-r06_f8w}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_f8.py -m gpu -x -q -s --timeout 180 --timeout-method thread \
    > gpurun_out/$tag/test_f8.log 2>&1 || { tail -40 gpurun_out/$tag/test_f8.log; exit 1; }
tail -2 gpurun_out/$tag/test_f8.log; grep "bf16f8w GEMM" gpurun_out/$tag/test_f8.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_model.py -m gpu -x -q -s --timeout 300 --timeout-method thread \
    -k "bf16f8 or knob" > gpurun_out/$tag/test_model.log 2>&1 || { tail -40 gpurun_out/$tag/test_model.log; exit 1; }
tail -2 gpurun_out/$tag/test_model.log; grep "ViT-B/16 bf16f8\|C1 \|N=290" gpurun_out/$tag/test_model.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 || { tail -20 gpurun_out/$tag/smoke.log; exit 1; }
tail -1 gpurun_out/$tag/smoke.log
for r in 1 2; do
  for q in weight no yes; do
    timeout -k 10 300 python3 bench.py --dtype bf16f8 --split-qkv $q --steps 10 --warmup 3 --no-secondary --no-evidence \
        --no-cpu-baseline > gpurun_out/$tag/bench_${q}_$r.json 2>/dev/null || exit 1
    echo "bf16f8 qkv=$q $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${q}_$r.json'));print(d['value'], d['ms_per_step'], d['parity']['logits_max_abs'], d['config'].get('knob_qkv'))")"
  done
done
