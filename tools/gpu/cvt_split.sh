set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/cvs
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "wgrad or linear" > gpurun_out/cvs/tests.log 2>&1
timeout -k 10 300 python -u tools/cvt_bench.py --no-torch > gpurun_out/cvs/cvt.json 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/cvs/vit.json 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/cvs/prof -o run --output-format csv -- python3 tools/cvt_bench.py --no-torch --steps 5 --warmup 2 > gpurun_out/cvs/prof.log 2>&1
