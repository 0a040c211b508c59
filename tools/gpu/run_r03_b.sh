# bench (+ secondary lines) + kernel summary, then GEMM rates and the CU-contention sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-r03_b}
mkdir -p gpurun_out/$tag
bash tools/gpu/bench.sh $tag || exit 1
timeout -k 10 240 python3 tools/gemm_bench.py 20 > gpurun_out/$tag/gemm_bench.txt 2>&1 || exit 1
timeout -k 10 400 python3 tools/contention.py 8 0 8 16 32 > gpurun_out/$tag/contention.jsonl 2>&1
