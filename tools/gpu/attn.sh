# attention kernels: parity tests + timing at the ViT-B/16 bs=256 shape (and N = 577)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k attention > gpurun_out/attn_test.log 2>&1 && \
timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 && \
timeout -k 10 120 python3 tools/attn_bench.py 64 577 16 >> gpurun_out/attn_bench.log 2>&1
