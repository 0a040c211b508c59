set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/apmc
timeout -k 10 60 rocprofv3 -L > gpurun_out/apmc/list.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/apmc/p1 -o run --output-format csv -- python3 tools/attn_one.py 3 > gpurun_out/apmc/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS -d $R/gpurun_out/apmc/p2 -o run --output-format csv -- python3 tools/attn_one.py 3 > gpurun_out/apmc/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $R/gpurun_out/apmc/p3 -o run --output-format csv -- python3 tools/attn_one.py 3 > gpurun_out/apmc/p3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/apmc/p4 -o run --output-format csv -- python3 tools/attn_one.py 3 > gpurun_out/apmc/p4.log 2>&1
