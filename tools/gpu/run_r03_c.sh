# bench (+ secondary lines, evidence legs) and its kernel summary; then the reserved-CU GEMM probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-r03_c}
mkdir -p gpurun_out/$tag
bash tools/gpu/bench.sh $tag || exit 1
timeout -k 10 200 python3 tools/reserve_probe.py > gpurun_out/$tag/reserve_probe.txt 2>&1
