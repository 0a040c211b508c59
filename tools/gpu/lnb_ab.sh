# LayerNorm backward grid-size A/B: tools/ln_bench.py for the in-tree build and variants/lnb*.so, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
  for v in base lnb256 lnb1024 lnb2048; do
    lib=""; [ $v != base ] && lib=transformer-stm_amd/variants/$v.so
    echo "$v: $(VITMI_LIB=$lib timeout -k 10 100 python3 tools/ln_bench.py 2>&1 | grep -v amdgpu | tr '\n' ' ')" || exit 1
  done
done
