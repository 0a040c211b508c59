# attention fwd/dQ stagger experiment: tools/attn_bench.py at the C3 shape for the in-tree build and
# variants/stag{1,2,3}.so, twice each.   bash tools/gpu/stag_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out/$tag
for i in 1 2; do
  for v in base stag1 stag2 stag3; do
    lib=""; [ $v != base ] && lib=transformer-stm_amd/variants/$v.so
    VITMI_LIB=$lib timeout -k 10 120 python3 tools/attn_bench.py 256 197 12 > gpurun_out/$tag/$v$i.log 2>&1 || exit 1
    echo "$v: $(grep seq gpurun_out/$tag/$v$i.log)"
  done
done
