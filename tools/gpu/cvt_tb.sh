set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/cvt gpurun_out/cvtb
timeout -k 10 400 python -u -m pytest tests/test_gpu_cvt.py tests/test_gpu_cvt_model.py -v --timeout 120 --timeout-method thread > gpurun_out/cvt/tests.log 2>&1
timeout -k 10 300 python -u tools/cvt_bench.py ${CVTB_ARGS:-} > gpurun_out/cvtb/bench.json 2> gpurun_out/cvtb/bench.err
cat gpurun_out/cvtb/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cvtb/prof -o run -- python3 tools/cvt_bench.py --no-torch --steps 5 --warmup 2 > gpurun_out/cvtb/prof.log 2>&1
