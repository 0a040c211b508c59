# Round 6: the single-pass attention backward: attention op tests, ViT-B model parity, the kernel
# timings (single-pass vs two-kernel vs streamed), the C3 step for policy 0 vs 3 (VITMI_ATTN_POLICY)
# and a rocprofv3 kernel summary of the default step.   bash tools/gpu/r06_attn.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=${1:-r06_attn}
mkdir -p gpurun_out/$tag
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py \
    -k "attention" > gpurun_out/$tag/test_ops.log 2>&1 || { tail -50 gpurun_out/$tag/test_ops.log; exit 1; }
tail -3 gpurun_out/$tag/test_ops.log
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py \
    -k "vit_b or c1 or determinism or bitwise" > gpurun_out/$tag/test_model.log 2>&1 || { tail -50 gpurun_out/$tag/test_model.log; exit 1; }
grep -E "logits max-abs|passed|failed" gpurun_out/$tag/test_model.log | tail -12
timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/$tag/attn_bench.txt 2>&1 || exit 1
cat gpurun_out/$tag/attn_bench.txt
for pol in 0 3 0 3; do
  timeout -k 10 200 python3 bench.py --attn-policy $pol --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
      --no-parity > gpurun_out/$tag/bench_p$pol.json 2>> gpurun_out/$tag/bench.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_p$pol.json'));print('policy $pol', d['value'], d['ms_per_step'], d['phases_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --no-parity --steps 5 --warmup 2 > gpurun_out/$tag/prof.log 2>&1 || exit 1
python3 tools/prof_summary.py "$(find gpurun_out/$tag/prof -name 'run_kernel_stats.csv' | head -1)" 7 > gpurun_out/$tag/summary.txt || exit 1
head -24 gpurun_out/$tag/summary.txt
