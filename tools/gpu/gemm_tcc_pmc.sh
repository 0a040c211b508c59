set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=gemm_tcc
mkdir -p gpurun_out/$tag
timeout -s KILL 60 rocprofv3 -L > gpurun_out/$tag/avail.txt 2>&1 || true
i=0
for set in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" "TA_BUSY_max TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/$tag/p$i -o run --output-format csv -- \
      python3 tools/gemm_pmc_one.py 2 > gpurun_out/$tag/p$i.log 2>&1 || echo "pass $i failed"
done
