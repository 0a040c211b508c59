# grouped tile order (VITMI_TILE_GM = 4 / 6 / 8 row panels per group) vs row-major (in-tree):
# GEMM shapes and the C3 step, 2 rounds; then the fc1 + GELU launch's L2 fetch (TCC_EA0_RDREQ via
# FETCH_SIZE) for base and gm8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_gm}
mkdir -p gpurun_out/$tag
timeout -k 10 300 env VITMI_LIB=$V/gm6.so python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    -k "gemm or linear or wgrad" tests > gpurun_out/$tag/tests_gm6.txt 2>&1 || { tail -30 gpurun_out/$tag/tests_gm6.txt; exit 1; }
tail -1 gpurun_out/$tag/tests_gm6.txt
for r in 1 2; do
  for v in base gm4 gm6 gm8; do
    L=""; [ $v != base ] && L=$V/$v.so
    VITMI_LIB=$L timeout -k 10 120 python3 tools/gemm_shapes.py > gpurun_out/$tag/shapes_${v}_$r.txt 2>&1 || exit 1
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['forward'], d['phases_ms']['backward'])") | $(grep -v amdgpu gpurun_out/$tag/shapes_${v}_$r.txt | awk '{print $(NF-3)}' | tr '\n' ' ')"
  done
done
