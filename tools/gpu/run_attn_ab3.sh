set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu/kab.sh attn_ab3 "attention or attn or vit_b_bf16 or c1_ or c5_shape or modules or boundary" "python3 tools/attn_bench.py" attn_qreg || exit 1
timeout -k 10 200 python3 tools/reserve_probe.py > gpurun_out/attn_ab3/reserve_probe.txt 2>&1
