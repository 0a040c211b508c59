# non-temporal store hints with the grouped tile order: VITMI_ST_MASK 3 (in-tree: gelu' aux + bf16
# C) vs 0 / 7 (+ fp32 C) / 15 (+ split-K slabs); the C3 step, 3 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_st}
mkdir -p gpurun_out/$tag
for r in 1 2 3; do
  for v in base st0 st7 st15; do
    L=""; [ $v != base ] && L=$V/$v.so
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['forward'], d['phases_ms']['backward'])")"
  done
done
