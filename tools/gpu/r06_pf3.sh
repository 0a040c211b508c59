# fused attention backward: where the next pair's loads go (pf 1 = all after phase 1, 0 = all after
# phase 2, 2 = dO image DMA after phase 2, 3 = register loads after phase 2): per-pair stamps + timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_pf3}
mkdir -p gpurun_out/$tag
for v in astamps astamps_pf0 astamps_pf2 astamps_pf3; do
  echo "== $v"; VITMI_LIB=$V/$v.so timeout -k 10 120 python3 tools/attn_fused_stamps.py > gpurun_out/$tag/$v.txt 2>&1 || exit 1
  cat gpurun_out/$tag/$v.txt | grep -v amdgpu.ids
done
for r in 1 2; do
  for v in base apf3; do
    L=""; [ $v != base ] && L=$V/$v.so
    echo "== $v $r"; VITMI_LIB=$L timeout -k 10 120 python3 tools/attn_bench.py 2>&1 | grep -v amdgpu.ids | head -2 || exit 1
  done
done
