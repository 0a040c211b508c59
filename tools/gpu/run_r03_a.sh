# Round-3 first evidence run: suite + bench (tools/gpu/run_r03.sh), then the GEMM rates and the
# one-GPU CU-contention sweep of the overlapped all-reduce (tools/contention.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-r03_a}
bash tools/gpu/run_r03.sh $tag || exit 1
timeout -k 10 240 python3 tools/gemm_bench.py 20 > gpurun_out/$tag/gemm_bench.txt 2>&1 || exit 1
timeout -k 10 400 python3 tools/contention.py 8 0 8 16 32 > gpurun_out/$tag/contention.jsonl 2>&1
