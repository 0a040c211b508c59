set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r05_overlap
timeout -k 10 180 python3 tools/overlap_probe.py 16 32 64 > gpurun_out/r05_overlap/probe.log 2>&1; rc=$?
cat gpurun_out/r05_overlap/probe.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/gemm_tn_pmc.sh r05_gemm_tn
cat gpurun_out/r05_gemm_tn/table.txt | head -80
