# weight-gradient L2 prefetch VITMI_WG_PFD K-steps ahead (4 / 6) vs none (in-tree): wgrad parity
# tests on each, GEMM shapes and the C3 step, 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_pfd}
mkdir -p gpurun_out/$tag
for v in pfd4 pfd6; do
  timeout -k 10 300 env VITMI_LIB=$V/$v.so python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
      -k "wgrad or linear" tests > gpurun_out/$tag/tests_$v.txt 2>&1 || { tail -30 gpurun_out/$tag/tests_$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/$tag/tests_$v.txt)"
done
for r in 1 2; do
  for v in base pfd4 pfd6; do
    L=""; [ $v != base ] && L=$V/$v.so
    VITMI_LIB=$L timeout -k 10 120 python3 tools/gemm_shapes.py > gpurun_out/$tag/shapes_${v}_$r.txt 2>&1 || exit 1
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['forward'], d['phases_ms']['backward'])") | $(grep -v amdgpu gpurun_out/$tag/shapes_${v}_$r.txt | tail -5 | head -4 | awk '{print $(NF-3)}' | tr '\n' ' ')"
  done
done
