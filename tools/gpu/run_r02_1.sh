set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r02_1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -s --timeout 180 --timeout-method thread > gpurun_out/r02_1/test.log 2>&1
echo "tests rc=$?" >> gpurun_out/r02_1/test.log
timeout -k 10 600 python3 bench.py > gpurun_out/r02_1/bench.json 2> gpurun_out/r02_1/bench.err
