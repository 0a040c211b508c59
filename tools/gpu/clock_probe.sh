# The GPU's shader clock while the fc1 GEMM runs back to back and while the C3 bench steps
# (rocm-smi samples beside the load).   bash tools/gpu/clock_probe.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out/$tag
echo "== idle"; rocm-smi --showclocks 2>&1 | grep -iE "sclk|mclk|fclk" | head -4
timeout -k 10 120 python3 tools/gemm_one.py fc1_store 40000 > gpurun_out/$tag/gemm.log 2>&1 &
pid=$!
sleep 12
for i in 1 2 3 4 5; do echo "== fc1 GEMM loop sample $i"; rocm-smi --showclocks --showpower 2>&1 | grep -iE "sclk|power" | head -3; sleep 1; done
wait $pid || exit 1
timeout -k 10 200 python3 bench.py --steps 400 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline > gpurun_out/$tag/bench.json 2>&1 &
pid=$!
sleep 20
for i in 1 2 3 4 5; do echo "== C3 bench sample $i"; rocm-smi --showclocks --showpower 2>&1 | grep -iE "sclk|power" | head -3; sleep 1; done
wait $pid || exit 1
grep -o '"value": [0-9.]*' gpurun_out/$tag/bench.json
