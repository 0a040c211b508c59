set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/dgbab
for F in 0 1 0 1 0 1; do
  echo "== F $F" >> gpurun_out/dgbab/bench.txt
  VITMI_FUSED_BIAS=$F timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/dgbab/bench.txt 2>&1
done
