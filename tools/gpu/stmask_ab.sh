# non-temporal hint per output class: aux + bf16 C (in-tree default) vs none (sm0) and vs
# + split-K partial slabs (sm11): tests on the in-tree build, GEMM shapes, 10-step bench, 2 rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu/kab.sh stmask2 "gemm or linear or aux_tiled or vit or modules or cvt or dropout or determin or boundary or wgrad" "python3 tools/gemm_bench.py 20" sm0 sm11
