# phase-offset experiments: fused attention backward start groups / mixed prefetch point, and gemm256
# start delays for the blocks with one tile fewer; isolated kernel tool + 10-step C3 bench, 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_desync}
mkdir -p gpurun_out/$tag
for r in 1 2; do
  for v in base adesync2 adesync4 apfmix gdesync gdesync1; do
    L=""; [ $v != base ] && L=$V/$v.so
    case $v in a*) tool=tools/attn_bench.py;; g*) tool=tools/gemm_shapes.py;; *) tool=tools/attn_bench.py;; esac
    VITMI_LIB=$L timeout -k 10 120 python3 $tool > gpurun_out/$tag/tool_${v}_$r.txt 2>&1 || exit 1
    if [ $v = base ]; then VITMI_LIB=$L timeout -k 10 120 python3 tools/gemm_shapes.py > gpurun_out/$tag/tool2_${v}_$r.txt 2>&1 || exit 1; fi
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
