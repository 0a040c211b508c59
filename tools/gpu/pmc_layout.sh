# SQ counters of the three GEMM layouts (one rocprofv3 --pmc pass per counter group; stops at
# the first failing pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/pmcl
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS \
    -d $R/gpurun_out/pmcl/p1 -o run --output-format csv -- python3 tools/gemm_layout_pmc.py > gpurun_out/pmcl/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM \
    -d $R/gpurun_out/pmcl/p2 -o run --output-format csv -- python3 tools/gemm_layout_pmc.py > gpurun_out/pmcl/p2.log 2>&1
