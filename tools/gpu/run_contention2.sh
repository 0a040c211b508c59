# CU-contention sweep after the split-K fix: torch-shaped side traffic and the RCCL-channel
# emulation (16 and 32 co-resident blocks), reserve_cus 0 / 16 / 32
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/cont2
timeout -k 10 300 python3 tools/contention.py 8 0 16 32 > gpurun_out/cont2/torch.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/contention.py 8 --emu 16 0 16 32 > gpurun_out/cont2/emu16.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/contention.py 8 --emu 32 0 16 32 48 > gpurun_out/cont2/emu32.jsonl 2>&1
