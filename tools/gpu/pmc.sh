# HBM traffic of one GEMM from two rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE cannot share
# a pass on gfx950):  bash tools/gpu/pmc.sh TAG [fc1_gelu|fc1_store|fc2_res]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=${1:-pmc}; which=${2:-fc1_gelu}
mkdir -p gpurun_out/$tag
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/$tag/fetch -o run --output-format csv -- \
    python3 tools/gemm_one.py $which 5 > gpurun_out/$tag/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/$tag/write -o run --output-format csv -- \
    python3 tools/gemm_one.py $which 5 > gpurun_out/$tag/write.log 2>&1 && \
python3 tools/pmc_traffic.py "$(find gpurun_out/$tag/fetch -name 'run_counter_collection.csv' | head -1)" \
    "$(find gpurun_out/$tag/write -name 'run_counter_collection.csv' | head -1)" gemm256_kernel \
    gpurun_out/$tag/traffic.json > gpurun_out/$tag/traffic.log 2>&1
