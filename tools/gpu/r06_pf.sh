# fused attention backward prefetch placement: stamps + attn_bench per variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
for v in astamps astamps_pf0 astamps_pf2; do echo "== $v"; VITMI_LIB=$V/$v.so timeout -k 10 120 python3 tools/attn_fused_stamps.py || exit 1; done
echo "== in-tree"; timeout -k 10 120 python3 tools/attn_bench.py || exit 1
for v in pf0 pf2; do echo "== $v"; VITMI_LIB=$V/$v.so timeout -k 10 120 python3 tools/attn_bench.py || exit 1; done
