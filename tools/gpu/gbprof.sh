set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/gbp
GEMM_BENCH_ONLY=square timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/gbp/gb.log 2>&1
bash tools/gpu/prof.sh s2
