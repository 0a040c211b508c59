set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/cvt
timeout -k 10 300 python -u -m pytest tests/test_gpu_cvt.py -x -v --timeout 120 --timeout-method thread > gpurun_out/cvt/tests.log 2>&1
