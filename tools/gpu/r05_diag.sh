# Round-5 first call: where the N=290 bf16 gradient error comes from, then attention counters
# at the ViT-B (C3) and ViT-L@384 (C5) shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r05_diag
timeout -k 10 300 python3 tools/diag_grad_precision.py > gpurun_out/r05_diag/grad.log 2>&1 || { tail -20 gpurun_out/r05_diag/grad.log; exit 1; }
cat gpurun_out/r05_diag/grad.log
bash tools/gpu/attn_pmc.sh r05_attn_c3 256 197 12 && bash tools/gpu/attn_pmc.sh r05_attn_c5 64 577 16
