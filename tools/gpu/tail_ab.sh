set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/tail
for r in 1 2; do
for T in 1 0; do
  echo "== TAIL $T" >> gpurun_out/tail/bench.txt
  VITMI_GEMM_TAIL=$T timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/tail/bench.txt 2>&1
done
done
