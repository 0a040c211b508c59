# single-pass attention backward: parity + determinism, kernel timing on/off, C3 bench A/B
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/fb
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "single_pass or attention_fwd_bwd" -x -q --timeout 120 --timeout-method thread > gpurun_out/fb/ops.log 2>&1
VITMI_ATTN_FUSED=0 timeout -k 10 120 python tools/attn_bench.py > gpurun_out/fb/attn0.log 2>&1
VITMI_ATTN_FUSED=1 timeout -k 10 120 python tools/attn_bench.py > gpurun_out/fb/attn1.log 2>&1
VITMI_ATTN_FUSED=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/fb/bench1.log 2>&1
VITMI_ATTN_FUSED=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/fb/bench0.log 2>&1
VITMI_ATTN_FUSED=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/fb/bench1b.log 2>&1
