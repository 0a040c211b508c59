# PMC passes over the attention fwd + bwd at the ViT-B shape with the single-pass backward
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp VITMI_ATTN_FUSED=1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/fpmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/fpmc/p1 -o run --output-format csv -- python3 tools/attn_one.py 3 > gpurun_out/fpmc/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS -d $R/gpurun_out/fpmc/p2 -o run --output-format csv -- python3 tools/attn_one.py 3 > gpurun_out/fpmc/p2.log 2>&1
