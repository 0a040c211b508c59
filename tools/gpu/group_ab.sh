set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/grp
for G in 1 4 8 16; do
  echo "== GROUP $G" >> gpurun_out/grp/gemm.txt
  VITMI_GEMM_GROUP=$G timeout -k 10 120 python tools/gemm_bench.py 20 >> gpurun_out/grp/gemm.txt 2>&1
done
for G in 1 8 1 8; do
  echo "== GROUP $G" >> gpurun_out/grp/bench.txt
  VITMI_GEMM_GROUP=$G timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/grp/bench.txt 2>&1
done
