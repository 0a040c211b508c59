# tail split for the K = 768 launches (VITMI_TAIL_MINK=8: qkv / proj / fc1 forward, proj dgrad; S <= 4
# or 2): GEMM shapes and the C3 step against the in-tree build, 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_tail}
mkdir -p gpurun_out/$tag
for r in 1 2; do
  for v in base tmink8 tmink8s2; do
    L=""; [ $v != base ] && L=$V/$v.so
    VITMI_LIB=$L timeout -k 10 120 python3 tools/gemm_shapes.py > gpurun_out/$tag/shapes_${v}_$r.txt 2>&1 || exit 1
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['forward'])") $(grep -E 'fwd|proj dgrad' gpurun_out/$tag/shapes_${v}_$r.txt | awk '{print $(NF-3)}' | tr '\n' ' ')"
  done
done
