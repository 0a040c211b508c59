# precision-knob checks: split / x3 op tests, the bf16x3 model tests (-s: logits error printed),
# then the bf16x3 bench line.   bash tools/gpu/x3_check.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-x3}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -k "split or x3 or attention or gelu" -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/ops.log 2>&1 || { tail -30 gpurun_out/$tag/ops.log; exit 1; }
tail -2 gpurun_out/$tag/ops.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_model.py -k "bf16x3" -x -q -s --timeout 300 --timeout-method thread > gpurun_out/$tag/model.log 2>&1 || { tail -30 gpurun_out/$tag/model.log; exit 1; }
grep -E "logits|worst|passed|failed" gpurun_out/$tag/model.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --dtype bf16x3 --steps 10 --warmup 3 > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || exit 1
cut -c1-300 gpurun_out/$tag/bench.json
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_cvt_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$tag/cvt.log 2>&1 || { tail -30 gpurun_out/$tag/cvt.log; exit 1; }
tail -2 gpurun_out/$tag/cvt.log
