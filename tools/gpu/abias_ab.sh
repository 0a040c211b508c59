set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/abias2
for r in 1 2; do
for F in "0 0" "1 0" "1 1" "0 1"; do
  set -- $F
  echo "== dgelu $1 qkv $2" >> gpurun_out/abias2/bench.txt
  VITMI_FUSED_BIAS=$1 VITMI_FUSED_QKV_BIAS=$2 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/abias2/bench.txt 2>&1
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/abias2/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/abias2/prof.log 2>&1
