# fused attention backward: odd workgroups started late (desync of the HBM bursts)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
for r in 1 2; do
  for v in base ds1 ds2 ds3; do
    L=""; [ $v != base ] && L=$V/$v.so
    echo "$v $r $(VITMI_LIB=$L timeout -k 10 120 python3 tools/attn_bench.py 2>/dev/null | head -1)"
  done
done
