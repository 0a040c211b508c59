set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/sls
timeout -k 10 400 python -u -m pytest tests/test_gpu_sls.py tests/test_gpu_cvt_model.py -v --timeout 120 --timeout-method thread > gpurun_out/sls/tests.log 2>&1
