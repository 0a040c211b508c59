# Round 6 check A: the changed GPU tests (world-2 comm leg over the functional stub, bf16f8 at large
# magnitudes), then the bench line with the per-line parity block and every secondary line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-r06_a}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
    tests/test_gpu_dp.py tests/test_gpu_f8.py -s > gpurun_out/$tag/test.log 2>&1 || { tail -40 gpurun_out/$tag/test.log; exit 1; }
grep -E "passed|failed|world-2 stub|bf16f8 GEMM" gpurun_out/$tag/test.log | tail -20
timeout -k 10 700 python3 bench.py --no-evidence > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { tail -20 gpurun_out/$tag/bench.err; exit 1; }
python3 - <<PY
import json
d = json.load(open("gpurun_out/$tag/bench.json"))
print(d["value"], d["ms_per_step"], d["phases_ms"], d.get("parity"))
for k, v in d.get("secondary", {}).items():
    print(k, v.get("value"), v.get("ms_per_step"), v.get("optimizer_ms"), v.get("parity", v.get("error")))
PY
