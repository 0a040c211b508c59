# tile-native gelu' (VITMI_EPI_AUX_TILED): the GPU tests it touches, GEMM shapes, a 10-step bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/tiled2
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "gemm or linear or aux_tiled or vit or modules or cvt or dropout or determin or boundary or sls" -x -q --timeout 120 --timeout-method thread > gpurun_out/tiled2/test.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/gemm_bench.py 20 > gpurun_out/tiled2/tool.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 10 --warmup 3 > gpurun_out/tiled2/step.log 2>&1
