set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/gpmc
for m in NT TN NN; do
  timeout -k 10 60 python3 tools/gemm_layout.py $m 10 >> gpurun_out/gpmc/time.txt 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/gpmc/${m}1 -o run --output-format csv -- python3 tools/gemm_layout.py $m 2 > gpurun_out/gpmc/${m}1.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS -d $R/gpurun_out/gpmc/${m}2 -o run --output-format csv -- python3 tools/gemm_layout.py $m 2 > gpurun_out/gpmc/${m}2.log 2>&1
done
cat gpurun_out/gpmc/time.txt
