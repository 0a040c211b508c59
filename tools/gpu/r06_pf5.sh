# fused attention backward: the next pair's O rows right after delta (pf 5) vs all loads after phase 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_pf5}
mkdir -p gpurun_out/$tag
for v in astamps_pf5 astamps_pf6 astamps_pf7; do
  echo "== $v"; VITMI_LIB=$V/$v.so timeout -k 10 120 python3 tools/attn_fused_stamps.py > gpurun_out/$tag/$v.txt 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/$tag/$v.txt
done
for r in 1 2; do
  for v in base apf5 apf6 apf7; do
    L=""; [ $v != base ] && L=$V/$v.so
    echo "== $v $r"; VITMI_LIB=$L timeout -k 10 120 python3 tools/attn_bench.py 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "step $v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
