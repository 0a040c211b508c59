# forward attention: K / V staged in 64-key chunks with the key loop starting on each as it lands
# (VITMI_FWD_CHUNKS=1, in-tree) vs the whole image first (fwdc0); attention tests first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
V=$PWD/transformer-stm_amd/variants
tag=${1:-r06_fwdc}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "attention or attn" tests \
    > gpurun_out/$tag/tests.txt 2>&1 || { tail -30 gpurun_out/$tag/tests.txt; exit 1; }
tail -2 gpurun_out/$tag/tests.txt
for r in 1 2; do
  for v in base fwdc0; do
    L=""; [ $v != base ] && L=$V/$v.so
    echo "== $v $r"; VITMI_LIB=$L timeout -k 10 120 python3 tools/attn_bench.py 2>&1 | grep -v amdgpu.ids | head -3 || exit 1
    VITMI_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
        --no-parity > gpurun_out/$tag/bench_${v}_$r.json 2>/dev/null || exit 1
    echo "step $v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
