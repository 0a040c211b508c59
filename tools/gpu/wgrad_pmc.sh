# Counters of the ViT-B weight-gradient GEMMs, one shape per process (verdict r04 item 4).
#   bash tools/gpu/wgrad_pmc.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$PWD
tag=${1:-wgrad_pmc}
mkdir -p gpurun_out/$tag
for shp in fc1 fc2 qkv proj; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/$shp/kt -o run --output-format csv -- \
      python3 tools/wgrad_pmc_one.py $shp 4 > gpurun_out/$tag/$shp.kt.log 2>&1 || exit 1
  i=0
  for set in "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "FETCH_SIZE TA_BUSY_max TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $set -d $R/gpurun_out/$tag/$shp/p$i -o run --output-format csv -- \
        python3 tools/wgrad_pmc_one.py $shp 2 > gpurun_out/$tag/$shp.p$i.log 2>&1 || echo "$shp pass $i failed"
  done
  echo "== $shp" >> gpurun_out/$tag/table.txt
  grep gemm256 gpurun_out/$tag/$shp/kt/run_kernel_stats.csv >> gpurun_out/$tag/table.txt || true
  python3 tools/pmc_table.py gpurun_out/$tag/$shp gemm256 >> gpurun_out/$tag/table.txt
done
