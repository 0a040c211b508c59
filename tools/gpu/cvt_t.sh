set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/cvt
timeout -k 10 400 python -u -m pytest ${CVT_TESTS:-tests/test_gpu_cvt.py tests/test_gpu_cvt_model.py} -v --timeout 120 --timeout-method thread > gpurun_out/cvt/tests.log 2>&1
