set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/side
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/side/tests.log 2>&1
VITMI_WGRAD_STREAM=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/side/bench_s0.log 2>&1
VITMI_WGRAD_STREAM=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/side/bench_s1.log 2>&1
VITMI_WGRAD_STREAM=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/side/bench_s0b.log 2>&1
VITMI_WGRAD_STREAM=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/side/bench_s1b.log 2>&1
