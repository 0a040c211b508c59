set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/slsb
timeout -k 10 500 python -u tools/sls_bench.py --frames 4000 --epochs 3 > gpurun_out/slsb/bench.json 2> gpurun_out/slsb/bench.err
cat gpurun_out/slsb/bench.json
