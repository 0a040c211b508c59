# TN vs NN main-loop counters at 8192^3 (one rocprofv3 --pmc pass per set; kernel-trace timing
# of the same launches first).   bash tools/gpu/gemm_tn_pmc.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=${1:-gemm_tn}
mkdir -p gpurun_out/$tag
timeout -s KILL 60 rocprofv3 -L > gpurun_out/$tag/avail.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/kt -o run --output-format csv -- \
    python3 tools/gemm_pmc_8k.py 3 > gpurun_out/$tag/kt.log 2>&1 || exit 1
i=0
for set in "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "TA_BUSY_max TA_ADDR_STALLED_BY_TC_CYCLES_sum FETCH_SIZE" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set -d $R/gpurun_out/$tag/p$i -o run --output-format csv -- \
      python3 tools/gemm_pmc_8k.py 2 > gpurun_out/$tag/p$i.log 2>&1 || echo "pass $i ($set) failed"
done
python3 tools/pmc_table.py gpurun_out/$tag gemm256 > gpurun_out/$tag/table.txt
grep -i "latency" gpurun_out/$tag/avail.txt | head -40 > gpurun_out/$tag/latency_counters.txt || true
