# RCCL-channel emulation with real traffic (16 loads in flight per thread), reserve sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/cont3
timeout -k 10 300 python3 tools/contention.py 8 --emu 16 0 16 32 > gpurun_out/cont3/emu16.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/contention.py 8 --emu 32 0 16 32 48 > gpurun_out/cont3/emu32.jsonl 2>&1
