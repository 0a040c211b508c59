set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/abias
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -v --timeout 120 --timeout-method thread -k "attention or model or block or fused" > gpurun_out/abias/tests.log 2>&1
for F in 0 1 0 1; do
  echo "== F $F" >> gpurun_out/abias/bench.txt
  VITMI_FUSED_BIAS=$F timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/abias/bench.txt 2>&1
done
