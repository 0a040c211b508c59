# column-panel groups as the outermost tile order (VITMI_TILE_NG=2: XCDs 0-3 take the first half of
# the columns, 4-7 the second) with GM 6 / 4 / 8 vs the in-tree order (GM 6, NG 1): GEMM parity
# tests on ng2gm6, GEMM shapes and the C3 step, 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_ng}
mkdir -p gpurun_out/$tag
timeout -k 10 300 env VITMI_LIB=$V/ng2gm6.so python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    -k "gemm or linear or wgrad" tests > gpurun_out/$tag/tests_ng2gm6.txt 2>&1 || { tail -30 gpurun_out/$tag/tests_ng2gm6.txt; exit 1; }
tail -1 gpurun_out/$tag/tests_ng2gm6.txt
for r in 1 2; do
  for v in base ng2gm6 ng2gm4 ng2gm8; do
    L=""; [ $v != base ] && L=$V/$v.so
    VITMI_LIB=$L timeout -k 10 120 python3 tools/gemm_shapes.py > gpurun_out/$tag/shapes_${v}_$r.txt 2>&1 || exit 1
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['forward'], d['phases_ms']['backward'])") | $(grep -v amdgpu gpurun_out/$tag/shapes_${v}_$r.txt | head -8 | awk '{print $(NF-3)}' | tr '\n' ' ')"
  done
done
