set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/opt
timeout -k 10 300 python -u -m pytest tests/test_optim.py tests/test_gpu_model.py -x -v --timeout 120 --timeout-method thread > gpurun_out/opt/tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/opt/bench_vitmi.json 2> gpurun_out/opt/bench_vitmi.err
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --optimizer torch > gpurun_out/opt/bench_torch.json 2> gpurun_out/opt/bench_torch.err
cat gpurun_out/opt/bench_vitmi.json gpurun_out/opt/bench_torch.json
