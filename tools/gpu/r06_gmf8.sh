# tile-group size for the bf16f8 line (F8 GEMM rows are 2K wide, so a row panel is twice the bytes)
# and for C5: GM 3 / 4 / 8 vs the in-tree 6, 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_gmf8}
mkdir -p gpurun_out/$tag
for r in 1 2; do
  for v in base gm3 gm4 gm8; do
    L=""; [ $v != base ] && L=$V/$v.so
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --config c3 --dtype bf16f8 --steps 10 --warmup 3 --no-secondary --no-evidence \
        --no-cpu-baseline --no-parity > gpurun_out/$tag/f8_${v}_$r.json 2>/dev/null || exit 1
    VITMI_LIB=$L timeout -k 10 300 python3 bench.py --config c5 --steps 6 --warmup 2 --no-secondary --no-evidence \
        --no-cpu-baseline --no-parity > gpurun_out/$tag/c5_${v}_$r.json 2>/dev/null || exit 1
    echo "$v $r f8 $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/f8_${v}_$r.json'));print(d['value'], d['phases_ms']['forward'])") c5 $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/c5_${v}_$r.json'));print(d['value'], d['phases_ms']['forward'])")"
  done
done
