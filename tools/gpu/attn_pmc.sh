# Counters of the bf16 attention kernels (fwd, dQ, dK/dV) at one shape, one rocprofv3 --pmc pass
# per set:  bash tools/gpu/attn_pmc.sh TAG [B N H]   (default ViT-B/16 bs 256: 256 197 12)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=${1:-attn_pmc}; shift
mkdir -p gpurun_out/$tag
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" \
           "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/$tag/p$i -o run --output-format csv -- \
      python3 tools/attn_one.py 3 "$@" > gpurun_out/$tag/p$i.log 2>&1 || exit 1
done
python3 tools/pmc_table.py gpurun_out/$tag attn > gpurun_out/$tag/table.txt
