# BASELINE config 5 (ViT-L/16 384px, N = 577): parity tests, bench line, kernel stats
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -k c5 -x -v --timeout 300 --timeout-method thread > gpurun_out/c5/tests.log 2>&1
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/c5/bench.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5/prof -o run --output-format csv -- python3 bench.py --config c5 --steps 5 --warmup 2 > gpurun_out/c5/prof.log 2>&1
